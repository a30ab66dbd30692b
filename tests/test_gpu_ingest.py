"""GPU parity of the on-device ingest: dc:31-34 column nnz scan and
dc:48-59 partition + standardisation (ingest.hip), through the C ABI, against the oracle's
host restatement (oracle/dc_oracle.py preprocess / partition / standardize).

Bars: nnz counts bit-exact (integer work).  Yd within 1e-13 relative (fp64; the device sums
rows in a different order from NumPy's pairwise mean/var); a sweep started from the device
Yd matches the oracle chain to the parity bar of test_gpu_parity (1e-10).
"""
import numpy as np
import pytest

import oracle
from helpers import STATE_CMP, make_case, rel_err, stacked_draws, state_dict
from oracle import dc_oracle as F

pytestmark = pytest.mark.gpu

YD_TOL = 1e-13
TOL = 1e-10


@pytest.mark.parametrize("n,p", [(1, 5), (37, 130), (64, 64), (1000, 515)])
def test_count_nonzero_columns_bit_exact(dcfm, n, p):
    r = np.random.default_rng(n * 7919 + p)
    Y = r.standard_normal((n, p))
    Y[:, ::7] = 0.0                                   # zero columns (dc:31-38)
    Y[:, 3 % p] = -0.0                                # nnz(-0) == 0
    if p > 10:
        Y[n // 2, 10] = np.nan                        # NaN counts as non-zero in nnz
        Y[:, 11] = 0.0
        Y[n - 1, 11] = 1e-300                         # one tiny non-zero entry
    got = dcfm.count_nonzero_columns(Y)
    want = np.count_nonzero(Y, axis=0).astype(np.int32)
    np.testing.assert_array_equal(got, want)


CASES = {
    # name: (n, p_raw, g, K, zero_cols)
    "basic": (40, 48, 4, 5, 0),
    "ragged_n_P": (37, 57, 3, 7, 0),          # n, P not multiples of 16 / 32
    "zero_cols": (45, 66, 4, 5, 2),           # dc:31-38 removes 2 columns -> P = 16
    "g1": (25, 20, 1, 4, 0),
    "many_shards": (20, 96, 12, 3, 0),
    "wide_P": (130, 400, 2, 40, 0),           # P = 200 spans 7 column tiles, n > 64 rows
    "long_n": (2100, 40, 2, 3, 0),            # n > 2,048: k_colstats' three-pass path
}


def _ingest(dcfm, c, smp, s0=0, gl=None):
    gl = c["g"] if gl is None else gl
    cols = dcfm.shard_columns(c["keep"], c["init"].varind, c["P"], s0, gl)
    return smp.set_data_raw(c["Y"], cols)


@pytest.mark.parametrize("name", list(CASES))
def test_set_data_raw_matches_host_standardisation(dcfm, name):
    n, p, g, K, z = CASES[name]
    c = make_case(n, p, g, K, zero_cols=z)
    smp = dcfm.Sampler(c["n"], c["P"], g, K, c["rho"], 0, 1, 1, inject_draws=True)
    try:
        sd, ms = _ingest(dcfm, c, smp)
        Yd = smp.get_data()
    finally:
        smp.close()
    assert rel_err(Yd, c["Yd"]) < YD_TOL
    Yk = c["Y"][:, c["keep"]]
    sd_ref = F.partition(Yk, g, c["init"].varind).std(axis=0, ddof=1)      # P x g
    assert rel_err(sd, sd_ref) < YD_TOL
    assert ms > 0.0


def test_zero_cols_rejected_in_preprocess_device(dcfm):
    """dc:41: P = p/g must be an integer after the zero columns are dropped."""
    Y, _ = oracle.synth.make_data(30, 40, k0=4, zero_cols=1)      # kept p = 39 -> not divisible by 4
    with pytest.raises(ValueError):
        dcfm.preprocess_device(Y, 4, 8)
    n, p, P, K, keep = dcfm.preprocess_device(make_case(30, 42, 4, 2, zero_cols=2)["Y"], 4, 8)
    assert (n, p, P, K) == (30, 40, 10, 2) and keep.size == 40


def test_constant_column_is_an_error(dcfm):
    """Q13: a constant non-zero column has zero variance; dc:59 would divide by zero."""
    c = make_case(30, 40, 4, 3)
    c["Y"][:, c["keep"][c["init"].varind[5]]] = 2.5
    smp = dcfm.Sampler(c["n"], c["P"], 4, 3, c["rho"], 0, 1, 1, inject_draws=True)
    try:
        with pytest.raises(dcfm.DcfmError) as ei:
            _ingest(dcfm, c, smp)
        assert ei.value.code == 1
        bad = np.array(dcfm.shard_columns(c["keep"], c["init"].varind, c["P"], 0, 4))
        bad[0] = c["Y"].shape[1]                    # out-of-range column index
        with pytest.raises(dcfm.DcfmError):
            smp.set_data_raw(c["Y"], bad)
    finally:
        smp.close()


@pytest.mark.parametrize("name", ["ragged_n_P", "zero_cols", "wide_P"])
def test_sweep_from_device_ingest_matches_oracle(dcfm, name):
    """yy (the residual-SS identity's input) is formed by the ingest kernel: the chain must
    still match the oracle started from the host-standardised Yd."""
    n, p, g, K, z = CASES[name]
    c = make_case(n, p, g, K, zero_cols=z)
    N = 3
    smp = dcfm.Sampler(c["n"], c["P"], g, K, c["rho"], 0, N, 1, inject_draws=True)
    try:
        _ingest(dcfm, c, smp)
        smp.set_state(state_dict(c["st"]))
        smp.set_draws(stacked_draws(c["src"], 1, N), 1, N)
        smp.run(1, N)
        got = smp.get_state()
        S = smp.get_sigma()
    finally:
        smp.close()
    ref = c["st"].copy()
    Sref = F.run_chain(c["Yd"], ref, c["rho"], c["hyper"], c["src"].iteration, 1, N, 0, N, 1)
    for f in STATE_CMP:
        e = rel_err(got[f], getattr(ref, f))
        assert e < TOL, f"{f} rel err {e:.3e}"
    assert rel_err(S, Sref) < TOL


def test_divideconquer_device_ingest_equals_host_ingest(dcfm):
    """The public entry point (dc:1) both ways, same injected draws: identical Sigmaout."""
    c = make_case(36, 50, 4, 3, zero_cols=2)
    N = 4
    draws = stacked_draws(c["src"], 1, N)
    out = []
    for dev in (True, False):
        S, info = dcfm.divideconquer(c["Y"], 4, 12, 1, 3, 1, c["rho"], init_draws=c["init"], iter_draws=draws,
                                     return_info=True, device_ingest=dev)
        out.append(S)
        assert info["p"] == 48 and info["P"] == 12
    assert rel_err(out[0], out[1]) < TOL


def test_two_ranks_ingest_their_own_shards(dcfm):
    """Each rank gathers only its shards' columns (shard_columns with s0 = rank * g_local)."""
    c = make_case(33, 72, 6, 3)
    gl = 3
    for r in range(2):
        smp = dcfm.Sampler(c["n"], c["P"], 6, 3, c["rho"], 0, 1, 1, nranks=2, rank=r, inject_draws=True)
        try:
            _ingest(dcfm, c, smp, s0=r * gl, gl=gl)
            Yd = smp.get_data()
        finally:
            smp.close()
        assert rel_err(Yd, c["Yd"][:, :, r * gl:(r + 1) * gl]) < YD_TOL


def test_ingest_c3_size_rates(dcfm):
    """c3-sized raw matrix (n = 1,000, p = 19,968): both ingest kernels run and report
    device times; the achieved HBM rates are printed (algorithmic bytes in DESIGN.md)."""
    n, g, P, K = 1000, 64, 312, 30
    p = g * P
    r = np.random.default_rng(5)
    Y = r.standard_normal((n, p))
    nnz, ms_nnz = dcfm.count_nonzero_columns(Y, return_ms=True)
    assert (nnz == n).all()
    varind = r.permutation(p)
    smp = dcfm.Sampler(n, P, g, K, 0.5, 0, 1, 1, inject_draws=True)
    try:
        sd, ms_std = smp.set_data_raw(Y, dcfm.shard_columns(np.arange(p), varind, P, 0, g))
        sd2, ms_std2 = smp.set_data_raw(Y, dcfm.shard_columns(np.arange(p), varind, P, 0, g))
        Yd = smp.get_data()
    finally:
        smp.close()
    j = varind[:P * 2]
    ref = (Y[:, j] - Y[:, j].mean(0)) / Y[:, j].std(0, ddof=1)
    assert rel_err(Yd[:, :, :2].reshape(n, -1, order="F"), ref) < YD_TOL
    b = 8.0 * n * p
    print(f"\nk_nnz_cols {ms_nnz * 1e3:.1f} us ({b / ms_nnz / 1e6:.0f} GB/s); "
          f"k_stdize {min(ms_std, ms_std2) * 1e3:.1f} us ({2 * b / min(ms_std, ms_std2) / 1e6:.0f} GB/s, "
          "read + write)")


def test_ingest_c5_size_sampled_columns(dcfm):
    """c5's full shape (n = 2,000, p = 100,096 = 391 x 256: 1.6 GB raw, > 2^31 elements of
    index space in the flattened input): nnz scan and standardise, checked on 96 sampled
    output columns against the host formula (size-independent per-column property)."""
    n, g, P, K = 2000, 256, 391, 30
    p = g * P
    r = np.random.default_rng(11)
    Y = np.empty((n, p), order="F")
    for c0 in range(0, p, 8192):                      # chunked fill keeps host peaks low
        c1 = min(p, c0 + 8192)
        Y[:, c0:c1] = r.standard_normal((n, c1 - c0)) * 2.0 + 0.5
    Y[:, 77] = 0.0
    nnz = dcfm.count_nonzero_columns(Y)
    assert nnz[77] == 0 and (np.delete(nnz, 77) == n).all()
    keep = np.flatnonzero(nnz != 0)                   # p - 1 kept: ingest the first p - 1 + a repeat
    cols_all = np.concatenate([keep, keep[:1]])       # P*g indices (any columns may repeat)
    varind = r.permutation(p)
    smp = dcfm.Sampler(n, P, g, K, 0.5, 0, 1, 1, inject_draws=True)
    try:
        sd, _ = smp.set_data_raw(Y, dcfm.shard_columns(cols_all, varind, P, 0, g))
        Yd = smp.get_data()
    finally:
        smp.close()
    pick = r.choice(p, size=96, replace=False)
    for q in pick:
        m, j = divmod(q, P)
        col = cols_all[varind[q]]
        x = Y[:, col]
        want = (x - x.mean()) * (1.0 / np.sqrt(x.var(ddof=1)))
        assert rel_err(Yd[:, j, m], want) < YD_TOL
        assert abs(sd[j, m] - x.std(ddof=1)) < 1e-12 * x.std(ddof=1)
