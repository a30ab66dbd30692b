"""Dev: ltphase instrumentation on the 4-waves/SIMD build."""
import subprocess, sys
subprocess.run([sys.executable, "tools/patches/ltphase.py", sys.argv[1]], check=True)
subprocess.run([sys.executable, "tools/patches/lt4.py", sys.argv[1]], check=True)
