"""A/B: kernels_wide.hip as committed (HEAD), the rest of the tree as is."""
import subprocess, sys, pathlib
src = subprocess.run(["git", "show", "HEAD:a-divide-and-conquer-strategy-for-high-dimensional-bayesian-factor-models_amd/csrc/kernels_wide.hip"],
                     check=True, capture_output=True, text=True).stdout
(pathlib.Path(sys.argv[1]) / "kernels_wide.hip").write_text(src)
