#!/bin/bash
# round 6: predict's table form (dl_embed_fwd_gtab + dl_gemm_s3_nt_gather_tab: the rows' offsets
# resolved by the lookup, staged by the layer) against the id form (fused) — gather tests, the
# front alone by mode (uniform / Zipf, lookup + layer timed back to back),
# then the bench line's lookup block
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06y2
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_parity.py -k "gather or fused or lookup_without" > $O/pytest.log 2>&1 || exit $?
tail -2 $O/pytest.log
for d in uniform zipf; do
  for m in fused tab fm fmtab fused tab fm fmtab; do
    timeout -k 10 200 python -u scripts/lookup_bench.py $d 100 $m 2>/dev/null >> $O/lookup.txt || exit $?
  done
done
cat $O/lookup.txt
timeout -k 10 400 python -u bench.py --no-extra --no-cpu-baseline --steps 20 > $O/bench.json 2> $O/bench.err || exit $?
python - <<PY
import json
d = json.loads(open("$O/bench.json").read().strip().splitlines()[-1])
g = d["gather_north_star"]["lookup_alone"]
for k, f in (("uniform", g["fused"]), ("zipf", g.get("zipf", {}).get("fused"))):
    print(k, {x: f[x] for x in ("fm_lookup_us", "fwd_l0_gather_us", "fwd_l0_plain_us", "us", "frac", "lookup_plus_l0_us")},
          "id", {x: f["id_form"][x] for x in ("fm_lookup_us", "fwd_l0_gather_us", "us", "frac")})
print("ms", d["ms_per_step"])
PY
