"""A/B (timing only, wrong results): k_assemble cross tiles neither read nor write Sigma."""
import subprocess, sys
subprocess.run([sys.executable, "tools/patches/anoload.py", sys.argv[1]], check=True)
subprocess.run([sys.executable, "tools/patches/anostore.py", sys.argv[1]], check=True)
