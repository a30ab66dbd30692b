"""Dev A/B: the committed (HEAD) kernel sources in place of the working copy's."""
import subprocess, sys
for name in ("kernels.hip", "kernels_wide.hip", "dcfm_internal.h", "linalg.h", "tile_linalg.h", "dcfm.hip"):
    src = subprocess.check_output(["git", "show", "HEAD:a-divide-and-conquer-strategy-for-high-dimensional-bayesian-factor-models_amd/csrc/" + name])
    open(sys.argv[1] + "/" + name, "wb").write(src)
