"""CPU oracle for the divide-and-conquer factor-model Gibbs sweep.

TEST INFRASTRUCTURE ONLY.  Nothing in the product path (the HIP library under
``a-divide-and-conquer-strategy-for-high-dimensional-bayesian-factor-models_amd/``)
imports, links or calls this package.  Only ``tests/``, ``__graft_entry__.smoke()``
and the ``cpu_baseline`` leg of ``bench.py`` use it, and only as the checker /
the CPU baseline.

What it is: a from-scratch NumPy restatement of the reference MATLAB function
``divideconquer.m`` (the reference repo's only code file), following it line by
line, every quirk included.  Each function cites the
reference lines it restates as ``dc:L``.

PARITY STATUS: **parity unpinned.**  The reference is MATLAB; no MATLAB or
Octave exists in this container or on the GPU box, and the reference ships no
tests, fixtures or golden vectors.  The restatement is
cross-checked only against itself (faithful per-row loop vs vectorised form),
against closed-form conditionals (the Gaussian full conditionals the sweep
samples from) and against documented MATLAB semantics (``cholcov`` returns the
upper factor, ``var`` uses n-1, ``cumprod`` runs along the first non-singleton
dimension, ``gamrnd(a,b) = b.*randg(a)``).  The golden fixtures under
``tests/golden`` are produced by this restatement (script committed beside
them); they pin the HIP kernels, not MATLAB.
"""
from .draws import DrawSource, InitDraws, IterDraws, gamma_shapes
from .dc_oracle import (
    Hyper,
    SamplerState,
    preprocess,
    partition,
    standardize,
    initialise,
    gibbs_iteration,
    assemble_sample,
    run_chain,
    divideconquer,
    cholcov,
    matlab_cumprod_delta,
)
from . import vectorised
from . import synth

__all__ = [
    "DrawSource", "InitDraws", "IterDraws", "gamma_shapes", "Hyper", "SamplerState",
    "preprocess", "partition", "standardize", "initialise", "gibbs_iteration",
    "assemble_sample", "run_chain", "divideconquer", "cholcov",
    "matlab_cumprod_delta", "vectorised", "synth",
]
