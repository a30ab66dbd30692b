"""A/B: zdraw with one accumulator chain per mt (fewer registers -> 3 blocks per CU)."""
import sys
f = sys.argv[1] + "/kernels.hip"
s = open(f).read()
old = """    d4 zw[2], zx[2], ze[2], as[2];
#pragma unroll
    for (int mt = 0; mt < 2; ++mt) zw[mt] = zx[mt] = ze[mt] = d4{0.0, 0.0, 0.0, 0.0};"""
new = """    d4 az[2], as[2];
#pragma unroll
    for (int mt = 0; mt < 2; ++mt) az[mt] = d4{0.0, 0.0, 0.0, 0.0};"""
assert old in s; s = s.replace(old, new)
old = """                zw[mt] = mfma16x16x4(Ms[0][16 * mt + c][kk], we, zw[mt]);
                zx[mt] = mfma16x16x4(Ms[1][16 * mt + c][kk], xe, zx[mt]);
                ze[mt] = mfma16x16x4(Ms[2][16 * mt + c][kk], ee, ze[mt]);"""
new = """                az[mt] = mfma16x16x4(Ms[0][16 * mt + c][kk], we, az[mt]);
                az[mt] = mfma16x16x4(Ms[1][16 * mt + c][kk], xe, az[mt]);
                az[mt] = mfma16x16x4(Ms[2][16 * mt + c][kk], ee, az[mt]);"""
assert old in s; s = s.replace(old, new)
old = """    d4 az[2];
#pragma unroll
    for (int mt = 0; mt < 2; ++mt) {
        az[mt] = (zw[mt] + zx[mt]) + ze[mt];
#pragma unroll"""
new = """#pragma unroll
    for (int mt = 0; mt < 2; ++mt) {
#pragma unroll"""
assert old in s; s = s.replace(old, new)
s = s.replace("__global__ __launch_bounds__(ZTHREADS) __attribute__((amdgpu_waves_per_eu(4))) void k_zxchol(", "__global__ __launch_bounds__(ZTHREADS) __attribute__((amdgpu_waves_per_eu(6))) void k_zxchol(")
open(f, "w").write(s)
