"""The Wide&Deep drop-in's own loop at C5 shapes (bench.py dropin_fit) alone:
python scripts/dropin_bench.py [n_batches]   (default: the native-decoded pinned feed;
DLAMD_PINNED_FEED=0: pickle.loads + pageable staging on the loop's thread)."""
import json
import os
import sys
import types

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 12
r = bench.dropin_fit(types.SimpleNamespace(batch=65536), n_batches=n)
r["feed"] = os.environ.get("DLAMD_PINNED_FEED", "1")
print(json.dumps(r), flush=True)
