#!/bin/bash
# round 6: the table form made opt-in (DLAMD_GATHER_TAB=1) — the whole GPU suite, then the
# default bench line (its lookup block times the id form, the table form and both pairs)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06z2
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err || exit $?
python - <<PY
import json
d = json.loads(open("$O/bench.json").read().strip().splitlines()[-1])
g = d["gather_north_star"]["lookup_alone"]
for k, f in (("uniform", g["fused"]), ("zipf", g.get("zipf", {}).get("fused"))):
    t = f.get("table_form", {})
    print(k, "id", {x: f[x] for x in ("fm_lookup_us", "fwd_l0_gather_us", "fwd_l0_plain_us", "us", "frac", "pair_minus_plain_us", "frac_by_pair")},
          "tab", {x: t.get(x) for x in ("fm_lookup_us", "fwd_l0_gather_us", "us", "frac", "pair_minus_plain_us", "frac_by_pair")})
print("ms", d["ms_per_step"], "value", d["value"], {k: v.get("ms_per_step") for k, v in d["extra_workloads"].items() if isinstance(v, dict)})
PY
tail -1 $O/bench.err
