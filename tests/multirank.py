"""Launch the driver as `world` rank processes (torchrun's env contract, 127.0.0.1 rendezvous)."""
import json
import os
import socket
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
WORKER = os.path.join(REPO, "tests", "_cli_worker.py")


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def run_ranks(world, argv, out_dir, fake, timeout=300):
    """Returns ([counts per rank], [stdout per rank]).  Raises if any rank fails."""
    port = free_port()
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), LOCAL_RANK="0", LOCAL_WORLD_SIZE=str(world),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), PYTHONUNBUFFERED="1")
        out = os.path.join(str(out_dir), f"counts_rank{r}.json")
        procs.append((out, subprocess.Popen([sys.executable, WORKER, out, "1" if fake else "0", "--"] + list(argv),
                                            env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)))
    outs = []
    try:
        for _, p in procs:
            outs.append(p.communicate(timeout=timeout)[0])
    finally:
        for _, p in procs:
            if p.poll() is None:
                p.kill()
    for (_, p), o in zip(procs, outs):
        assert p.returncode == 0, f"rank failed ({p.returncode}):\n{o[-3000:]}"
    counts = [{k: tuple(v) for k, v in json.load(open(o)).items()} for o, _ in procs]
    return counts, outs
