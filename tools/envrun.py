"""Run a python script with extra environment variables, as a child process (for tools/gpu.sh's `py`
step, whose lines cannot carry an environment): python tools/envrun.py KEY=VAL ... script.py args"""
import os
import subprocess
import sys

env = dict(os.environ)
args = sys.argv[1:]
while args and "=" in args[0] and not args[0].endswith(".py"):
    k, v = args.pop(0).split("=", 1)
    env[k] = v
sys.exit(subprocess.run([sys.executable, "-u"] + args, env=env).returncode)
