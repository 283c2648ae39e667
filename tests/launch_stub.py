"""Stand-in rank for tests/test_launch.py: stops before any GPU call.

Rank 0 prints one JSON line with the rank env it saw (what bench.py's rank 0
prints is its one result line); other ranks print to stdout too, which the
launcher must keep off the relayed stream.  STUB_FAIL_RANK=r makes rank r
exit 3 after STUB_FAIL_AFTER seconds; STUB_HANG=1 makes the other ranks sleep
(as ranks blocked in a collective would) until the launcher stops them.
"""

import json
import os
import sys
import time

rank = int(os.environ["RANK"])
keys = ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT",
        "HSA_ENABLE_IPC_MODE_LEGACY")
env = {k: os.environ.get(k) for k in keys}
env["pid"] = os.getpid()
fail = os.environ.get("STUB_FAIL_RANK")
if fail is not None and int(fail) == rank:
    time.sleep(float(os.environ.get("STUB_FAIL_AFTER", "0")))
    sys.exit(3)
if rank == 0:
    print(json.dumps({"stub": True, "argv": sys.argv[1:], "env": env}), flush=True)
else:
    print(f"rank {rank} stdout", flush=True)
    with open(os.path.join(os.environ["STUB_DIR"], f"rank{rank}.json"), "w") as fh:
        json.dump(env, fh)
if os.environ.get("STUB_HANG") == "1":
    time.sleep(600)
