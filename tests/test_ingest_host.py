"""Host logic of the on-device ingest (no GPU): the column map handed to dcfm_set_data_raw
reproduces dc:36-54's Y(:, setdiff(...)) then Y(:, varind(block m)) gather, for every rank's
shard range."""
import numpy as np

import oracle
from oracle import dc_oracle as F


def test_shard_columns_reproduce_partition(dcfm):
    Y, _ = oracle.synth.make_data(25, 66, k0=3, zero_cols=2)
    g = 4
    Yk, n, p, P, K, keep = F.preprocess(Y, g, 8)
    varind = np.random.default_rng(1).permutation(p)
    Yd = F.partition(Yk, g, varind)                         # n x P x g
    for nranks in (1, 2, 4):
        gl = g // nranks
        for r in range(nranks):
            cols = dcfm.shard_columns(keep, varind, P, r * gl, gl)
            assert cols.dtype == np.int64 and cols.size == P * gl
            got = Y[:, cols].reshape(n, P, gl, order="F")
            np.testing.assert_array_equal(got, Yd[:, :, r * gl:(r + 1) * gl])
