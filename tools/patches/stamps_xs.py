import subprocess, sys
d = sys.argv[1]
subprocess.check_call([sys.executable, "tools/patches/stamps.py", d])
subprocess.check_call([sys.executable, "tools/patches/xsphase.py", d])
