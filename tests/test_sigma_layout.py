"""Sigma's tile-packed layout (dcfm_internal.h sig_off / sig_tile_off), checked on the host.

k_assemble writes each 128 x 128 tile in its accumulator order (wave, 16x16 MFMA tile, lane, the
lane's value pairs adjacent); k_sigma_pack and k_sigma_err read single elements through sig_off.
A tiny host program built from the library's own header checks that the two agree: sig_off maps
the stored elements (a >= b) of a rank's tile rows one-to-one into its block, and the element
k_assemble's lane (wave, u, v, g) holds sits exactly where sig_off says (dc:194-195 read-out).
No GPU: hipcc compiles the header for the host.
"""
import shutil
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
CSRC = ROOT / "a-divide-and-conquer-strategy-for-high-dimensional-bayesian-factor-models_amd" / "csrc"
HIPCC = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"

PROG = r"""
#include "dcfm_internal.h"
#include <cstdio>
#include <vector>
using namespace dcfm;
int main() {
    const int p = 300, T0 = 1, T1 = 3;               // a rank owning tile rows [1, 3): rows [128, 300)
    const size_t nt = (size_t)(tri(T1) - tri(T0));
    std::vector<int> seen(nt * ASM_TILE * ASM_TILE, 0);
    long long bad = 0, n = 0;
    for (int a = T0 * ASM_TILE; a < p && a < T1 * ASM_TILE; ++a)
        for (int b = 0; b <= a; ++b) {
            const size_t o = sig_off(a, b, T0);
            if (o >= seen.size() || seen[o]++) ++bad;
            ++n;
        }
    // k_assemble's lane view of tile (ti, tj): wave w = 2 (row half) + column half, lane (r, q)
    // holds rows q + 4g of 16-row tile u, column r of 16-column tile v
    long long mism = 0;
    for (int ti = T0; ti < T1; ++ti)
        for (int tj = 0; tj <= ti; ++tj) {
            const size_t base = (size_t)(tri(ti) - tri(T0) + tj) * ASM_TILE * ASM_TILE;
            for (int w = 0; w < 4; ++w)
                for (int lane = 0; lane < 64; ++lane)
                    for (int u = 0; u < 4; ++u)
                        for (int v = 0; v < 4; ++v)
                            for (int g = 0; g < 4; ++g) {
                                const int r = lane & 15, q = lane >> 4;
                                const int a = ti * ASM_TILE + (w >> 1) * 64 + 16 * u + q + 4 * g;
                                const int b = tj * ASM_TILE + (w & 1) * 64 + 16 * v + r;
                                const size_t o = base + sig_tile_off(u, v, g, w, lane);
                                if (a < p && b <= a && sig_off(a, b, T0) != o) ++mism;
                                // the pair (g, g ^ 1) of one lane is 16-byte adjacent
                                if ((g & 1) == 0 && sig_tile_off(u, v, g + 1, w, lane) != sig_tile_off(u, v, g, w, lane) + 1) ++mism;
                            }
        }
    std::printf("%lld %lld %lld\n", n, bad, mism);
    return 0;
}
"""


@pytest.mark.skipif(not Path(HIPCC).exists(), reason="hipcc not available")
def test_sig_off_matches_the_assembly_lane_layout(tmp_path):
    src = tmp_path / "layout.cpp"
    src.write_text(PROG)
    exe = tmp_path / "layout"
    subprocess.run([HIPCC, "-std=c++17", "-O1", "-I", str(CSRC), "-I", str(ROOT / "include"), str(src), "-o", str(exe)],
                   check=True, capture_output=True)
    n, bad, mism = map(int, subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split())
    assert n == sum(a + 1 for a in range(128, 300))   # every stored element of rows [128, 300)
    assert bad == 0, "sig_off is not one-to-one into the rank's block"
    assert mism == 0, "sig_off disagrees with k_assemble's accumulator order"
