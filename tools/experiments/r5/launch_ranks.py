"""Start N copies of a command as ranks RANK = 0..N-1 (WORLD_SIZE, LOCAL_RANK, MASTER_* set) and wait.
The parent never touches the GPU: each rank may itself be `rocprofv3 ... -- python ...` (the profiler
wraps the program it starts; no launcher re-execs under it).  '{rank}' in the command is replaced.

    python tools/experiments/r5/launch_ranks.py 2 -- rocprofv3 --kernel-trace --stats -d out/r{rank} -- python x.py
"""
import os
import socket
import subprocess
import sys

n = int(sys.argv[1])
cmd = sys.argv[sys.argv.index("--") + 1:]
s = socket.socket()
s.bind(("127.0.0.1", 0))
port = str(s.getsockname()[1])
s.close()
procs = []
for r in range(n):
    env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
               MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
    procs.append(subprocess.Popen([c.replace("{rank}", str(r)) for c in cmd], env=env))
codes = [p.wait() for p in procs]
sys.exit(next((c for c in codes if c), 0))
