"""`python tests/_bench_selflaunch_worker.py --gpus N ...` = `python bench.py --gpus N ...` with the stand-in engine
(tests/test_bench_dist.py): bench.main() with no torchrun environment starts N copies of this script as ranks
(bench.self_launch), each of which runs bench.main() again under the RANK / WORLD_SIZE / MASTER_* contract.
BENCH_SEEN_DIR: each rank writes the utterances its engine saw there; BENCH_FAIL_RANK: that rank exits with 3
before joining the process group (the launcher must stop the others)."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import bench  # noqa: E402
from tests._bench_dist_worker import StandInEngine  # noqa: E402


def factory(rank):
    if os.environ.get("BENCH_FAIL_RANK") == str(rank):
        sys.exit(3)
    eng = StandInEngine(rank)
    d = os.environ.get("BENCH_SEEN_DIR")

    class Recording:
        def __getattr__(self, k):
            return getattr(eng, k)

        def close(self):
            if d:
                json.dump(eng.seen, open(os.path.join(d, f"seen{rank}.json"), "w"))

    rec = Recording()
    return lambda cfg, B, N: rec


if __name__ == "__main__":
    sys.exit(bench.main(sys.argv[1:], engine_factory=factory, script=os.path.abspath(__file__)))
