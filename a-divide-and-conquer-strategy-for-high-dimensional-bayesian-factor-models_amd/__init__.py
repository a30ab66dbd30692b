"""dcfm_amd — MI355X-native hot path of the divide-and-conquer Bayesian factor model.

Drop-in for the iteration loop of the reference ``divideconquer.m`` (lines
90-197: per-shard Gibbs sweep + covariance assembly), behind the C ABI in
``include/dcfm.h``; HIP kernels for gfx950 live in ``csrc/``.

Import through the repo-root helper (the directory name has hyphens)::

    import __graft_entry__ as ge; dcfm = ge.load_package()
    Sigmaout = dcfm.divideconquer(Y, g, k, BURNIN, MCMC, thin, rho)
"""
from ._abi import DcfmError, load_library, EXPORTS, LIB_PATH
from .sampler import Hyper, Sampler, rng_fill, count_nonzero_columns, STATE_FIELDS
from . import diagnostics
from .driver import divideconquer, preprocess, preprocess_device, shard_columns, partition_standardize, initial_state, local_state, truth_factors, output_columns, unpermute_sigma

__all__ = [
    "DcfmError", "load_library", "EXPORTS", "LIB_PATH", "Hyper", "Sampler", "rng_fill",
    "STATE_FIELDS", "divideconquer", "preprocess", "partition_standardize", "initial_state",
    "local_state", "truth_factors", "output_columns", "unpermute_sigma", "count_nonzero_columns",
    "preprocess_device", "shard_columns", "diagnostics",
]
