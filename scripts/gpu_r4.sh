#!/bin/bash
# Round-4 GPU steps: bash scripts/gpu_r4.sh MODE TAG
#   quick   the GPU suite without the full-size trajectories, then C3 uniform and Zipf benches
#   full    the full-size trajectories (C2, C3 10 steps with the fp64 audit; C5; C4)
#   bench   the default bench line
MODE=$1
TAG=${2:-r4}
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
if [ "$MODE" = quick ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu --maxfail=8 -q -rf -p no:cacheprovider --timeout 300 --timeout-method thread \
    --deselect tests/test_gpu_fullsize.py --durations=10 > $OUT/pytest_quick.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -15 $OUT/pytest_quick.log; [ $rc -eq 0 ] || exit $rc
  timeout -k 10 300 python bench.py --workload c3 --no-extra --no-cpu-baseline --steps 10 > $OUT/c3.json 2> $OUT/c3.err
  rc=$?; echo "c3 rc=$rc"; [ $rc -eq 0 ] || { tail -5 $OUT/c3.err; exit $rc; }
  python scripts/bench_brief.py $OUT/c3.json
  timeout -k 10 300 python bench.py --workload c3 --dist zipf --no-extra --no-cpu-baseline --steps 10 > $OUT/c3z.json 2> $OUT/c3z.err
  rc=$?; echo "c3 zipf rc=$rc"; [ $rc -eq 0 ] || { tail -5 $OUT/c3z.err; exit $rc; }
  python scripts/bench_brief.py $OUT/c3z.json
  exit 0
fi
if [ "$MODE" = full ]; then
  export DLAMD_TEST_STATS=$OUT
  timeout -k 10 1100 python -u -m pytest tests/test_gpu_fullsize.py -x -v -rf -p no:cacheprovider --timeout 1000 \
    --timeout-method thread --durations=6 > $OUT/pytest_full.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -15 $OUT/pytest_full.log; exit $rc
fi
if [ "$MODE" = bench ]; then
  timeout -k 10 600 python bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err
  rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || { tail -5 $OUT/bench_default.err; exit $rc; }
  python scripts/bench_brief.py $OUT/bench_default.json
  exit 0
fi
if [ "$MODE" = trace ]; then
  # kernel timeline of the hipGraph steps (workload $3, default c2)
  WL=${3:-c2}
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/trace_$WL -o trace -- \
    python bench.py --no-extra --no-cpu-baseline --workload $WL --steps 10 --warmup 3 --age-steps 16 \
    > $OUT/trace_$WL.log 2>&1
  rc=$?; echo "trace rc=$rc"; [ $rc -eq 0 ] || { tail -5 $OUT/trace_$WL.log; exit $rc; }
  f=$(ls $OUT/trace_$WL/*kernel_trace.csv 2>/dev/null | head -1)
  [ -n "$f" ] || f=$(find $OUT/trace_$WL -name "*kernel_trace.csv" | head -1)
  python scripts/step_timeline.py "$f" > $OUT/timeline_$WL.txt && head -40 $OUT/timeline_$WL.txt
  exit 0
fi
if [ "$MODE" = hosttrace ]; then
  # kernels and HIP API calls of the hipGraph steps: host submission against the GPU at the boundary
  WL=${3:-c5}
  timeout -k 10 300 rocprofv3 --kernel-trace --hip-runtime-trace --output-format csv -d $OUT/htrace_$WL -o trace -- \
    python bench.py --no-extra --no-cpu-baseline --workload $WL --steps 10 --warmup 3 --age-steps 16 \
    > $OUT/htrace_$WL.log 2>&1
  rc=$?; echo "htrace rc=$rc"; [ $rc -eq 0 ] || { tail -5 $OUT/htrace_$WL.log; exit $rc; }
  k=$(find $OUT/htrace_$WL -name "*kernel_trace.csv" | head -1)
  a=$(find $OUT/htrace_$WL -name "*hip_api_trace.csv" | head -1)
  python scripts/host_timeline.py "$k" "$a" > $OUT/host_timeline_$WL.txt; rc=$?
  head -30 $OUT/host_timeline_$WL.txt; exit $rc
fi
if [ "$MODE" = s3d7 ]; then
  # the NT kernels' A pieces as contiguous 64-B half lines: the k-permuted planes (variant kp,
  # DL_S3_KPERM=1) through the s3 kernel and tower tests, then kernel times default / diag 7
  # (timing only) / kp, then C2 and C3 step A/B
  DLAMD_VARIANT=kp timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_parity.py -m gpu -q -rf \
    -k "s3 or split3 or deepfm_pipeline" -p no:cacheprovider --timeout 200 --timeout-method thread > $OUT/pytest_kp.log 2>&1
  rc=$?; echo "pytest kp rc=$rc: $(tail -1 $OUT/pytest_kp.log)"; [ $rc -eq 0 ] || { grep -E "^(FAILED|ERROR)" $OUT/pytest_kp.log; exit $rc; }
  for rep in 1 2; do
    for v in "" diag7 kp; do
      for c in fwd_l0 fwd_l1 dx_l1; do
        DLAMD_VARIANT=$v timeout -k 10 120 python scripts/s3_bench.py 30 t:$c 2>&1 | grep -v amdgpu.ids | sed "s/^/[${v:-default}] /" | tee -a $OUT/d7.txt || exit 1
      done
    done
  done
  bash scripts/gpu_ab_variant.sh ${TAG}_kp kp "" "" "c2 c3"
  exit $?
fi
if [ "$MODE" = pfmid ]; then
  # the step in two launches with the prefetch released between them: bit-identity, A/B, trace
  timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -rf -k prefetch_matches \
    -p no:cacheprovider --timeout 200 --timeout-method thread > $OUT/pytest_pfmid.log 2>&1
  rc=$?; echo "pytest rc=$rc: $(tail -1 $OUT/pytest_pfmid.log)"; [ $rc -eq 0 ] || { grep -E "^(FAILED|ERROR)" $OUT/pytest_pfmid.log; exit $rc; }
  for rep in 1 2 3; do
    cfgs="c5:0 c5:1 c2:0 c2:1"; [ $rep -eq 3 ] && cfgs="c3:0 c3:1"
    for cfg in $cfgs; do
      IFS=: read wl e <<< "$cfg"
      DLAMD_STEP_EVENTS=1 DLAMD_PF_MID=$e timeout -k 10 300 python bench.py --no-cpu-baseline --no-extra --workload $wl \
        --steps 20 --warmup 5 > $OUT/mid_${wl}_$e.json 2> $OUT/mid_${wl}_$e.err || { tail -5 $OUT/mid_${wl}_$e.err; exit 1; }
      python -c "
import json;d=json.loads(open('$OUT/mid_${wl}_$e.json').read().strip().splitlines()[-1])
print('$wl pf_mid=$e', d['ms_per_step'], 'host', d.get('host_submit_ms_per_step'), 'events', d.get('step_events'))"
    done
  done
  DLAMD_PF_MID=1 bash scripts/gpu_r4.sh trace ${TAG}_mid c5 && DLAMD_PF_MID=1 bash scripts/gpu_r4.sh trace ${TAG}_mid c2
  exit $?
fi
if [ "$MODE" = cores ]; then
  # the index build's kernels sized to share a CU with the forward NT GEMM block (LDS <= 43 KB,
  # VGPR <= 112): radix tiles of 14 / 12 rounds (and pre-materialised keys); sort tests per
  # variant, then step A/B on C2, C3, C5
  for v in r14 r12 r12pk; do
    DLAMD_VARIANT=$v timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_parity.py -m gpu -q -rf \
      -k "index or sort_unique or prefetch_matches" -p no:cacheprovider --timeout 200 --timeout-method thread > $OUT/pytest_$v.log 2>&1
    rc=$?; echo "pytest $v rc=$rc: $(tail -1 $OUT/pytest_$v.log)"; [ $rc -eq 0 ] || { grep -E "^(FAILED|ERROR)" $OUT/pytest_$v.log; exit $rc; }
  done
  for v in r14 r12 r12pk; do
    bash scripts/gpu_ab_variant.sh ${TAG}_$v $v "" "" "c2 c5 c3" || exit $?
  done
  exit 0
fi
if [ "$MODE" = rsbig ]; then
  # the size-chosen radix tile (12 rounds + pre-materialised keys from 2 M references) against the
  # previous single configuration (variant old): index / sort / prefetch / wdl tests, then A/B
  timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_parity.py tests/test_gpu_dropin.py -m gpu -q -rf \
    -k "index or sort_unique or prefetch or hot or wdl or multi_cate" -p no:cacheprovider --timeout 200 --timeout-method thread > $OUT/pytest_rs.log 2>&1
  rc=$?; echo "pytest rc=$rc: $(tail -1 $OUT/pytest_rs.log)"; [ $rc -eq 0 ] || { grep -E "^(FAILED|ERROR)" $OUT/pytest_rs.log; exit $rc; }
  bash scripts/gpu_ab_variant.sh ${TAG}_ab old "" "" "c5 c3 c2"
  exit $?
fi
if [ "$MODE" = stgap ]; then
  # what the per-step status read-back costs the boundary: read back every step vs (almost) never
  # (ring: the status written by the step's last kernel into pinned memory, DLAMD_STATUS_RING)
  timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -rf -k "bad_id" \
    -p no:cacheprovider --timeout 200 --timeout-method thread > $OUT/pytest_ring.log 2>&1
  rc=$?; echo "pytest rc=$rc: $(tail -1 $OUT/pytest_ring.log)"; [ $rc -eq 0 ] || { grep -E "^(FAILED|ERROR)" $OUT/pytest_ring.log; exit $rc; }
  for rep in 1 2; do
    for wl in c5 c2; do
      for cfg in 1:0 1000:0 1:1; do
        IFS=: read ev rg <<< "$cfg"
        DLAMD_STEP_EVENTS=1 DLAMD_STATUS_EVERY=$ev DLAMD_STATUS_RING=$rg timeout -k 10 300 python bench.py --no-cpu-baseline --no-extra \
          --workload $wl --steps 30 --warmup 5 > $OUT/st_${wl}_$ev$rg.json 2> $OUT/st_${wl}_$ev$rg.err || { tail -5 $OUT/st_${wl}_$ev$rg.err; exit 1; }
        python -c "
import json;d=json.loads(open('$OUT/st_${wl}_$ev$rg.json').read().strip().splitlines()[-1])
print('$wl status_every=$ev ring=$rg', d['ms_per_step'], 'host', d.get('host_submit_ms_per_step'), 'events', d.get('step_events'))"
      done
    done
  done
  exit 0
fi
if [ "$MODE" = hotfold ]; then
  # the hot-row chunk scan folded into pass 1's last block (variant nofold: its own launch)
  timeout -k 10 400 python -u -m pytest tests -m gpu -q -rf -k "hot or determin or lazy or prefetch or bad_id or zipf" \
    --deselect tests/test_gpu_fullsize.py -p no:cacheprovider --timeout 200 --timeout-method thread > $OUT/pytest_hot.log 2>&1
  rc=$?; echo "pytest rc=$rc: $(tail -1 $OUT/pytest_hot.log)"; [ $rc -eq 0 ] || { grep -E "^(FAILED|ERROR)" $OUT/pytest_hot.log; exit $rc; }
  timeout -k 10 300 python bench.py --workload c3 --dist zipf --no-extra --no-cpu-baseline --steps 10 > $OUT/c3z.json 2> $OUT/c3z.err || { tail -5 $OUT/c3z.err; exit 1; }
  python scripts/bench_brief.py $OUT/c3z.json
  bash scripts/gpu_ab_variant.sh ${TAG}_ab nofold "" "" "c2 c5"
  exit $?
fi
if [ "$MODE" = s3pf ]; then
  # the NT kernels' weight-fragment read distance (DL_S3_PF 1 default, variants pf2 / pf3)
  for v in pf2 pf3; do
    DLAMD_VARIANT=$v timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -q -rf -k "s3" \
      -p no:cacheprovider --timeout 200 --timeout-method thread > $OUT/pytest_$v.log 2>&1
    rc=$?; echo "pytest $v rc=$rc: $(tail -1 $OUT/pytest_$v.log)"; [ $rc -eq 0 ] || exit $rc
  done
  for rep in 1 2; do
    for v in "" pf2 pf3; do
      for c in fwd_l1 dx_l1; do
        DLAMD_VARIANT=$v timeout -k 10 120 python scripts/s3_bench.py 30 t:$c 2>&1 | grep -v amdgpu.ids | sed "s/^/[${v:-default}] /" | tee -a $OUT/pf.txt || exit 1
      done
    done
  done
  bash scripts/gpu_ab_variant.sh ${TAG}_pf2 pf2 "" "" "c2" && bash scripts/gpu_ab_variant.sh ${TAG}_pf3 pf3 "" "" "c2"
  exit $?
fi
if [ "$MODE" = pfmid2 ]; then
  # prefetch depth x release point (d1m0 = the default): step time and the event span / gap
  for rep in 1 2 3; do
    wls="c5 c2"; [ $rep -eq 3 ] && wls="c3"
    for wl in $wls; do
      for cfg in 1:0 2:1 2:0; do
        IFS=: read dp e <<< "$cfg"
        DLAMD_STEP_EVENTS=1 DLAMD_PF_DEPTH=$dp DLAMD_PF_MID=$e timeout -k 10 300 python bench.py --no-cpu-baseline --no-extra \
          --workload $wl --steps 30 --warmup 5 > $OUT/m2_${wl}_$dp$e.json 2> $OUT/m2_${wl}_$dp$e.err || { tail -5 $OUT/m2_${wl}_$dp$e.err; exit 1; }
        python -c "
import json;d=json.loads(open('$OUT/m2_${wl}_$dp$e.json').read().strip().splitlines()[-1])
print('$wl depth=$dp mid=$e', d['ms_per_step'], 'host', d.get('host_submit_ms_per_step'), 'events', d.get('step_events'))"
      done
    done
  done
  exit 0
fi
if [ "$MODE" = combo ]; then
  # quick, then an A/B of a library variant ($3) on C2 and C3
  bash scripts/gpu_r4.sh quick $TAG || exit $?
  bash scripts/gpu_ab_variant.sh ${TAG}_ab $3 "" "" "c2 c3"
  exit $?
fi
if [ "$MODE" = perf ]; then
  # step timelines of C2 and C5, then the replay A/B (paired vs single-element units)
  bash scripts/gpu_r4.sh trace $TAG c2 || exit $?
  bash scripts/gpu_r4.sh trace $TAG c5 || exit $?
  bash scripts/gpu_ab_variant.sh ${TAG}_rp rp1 "" "" "c2 c5" || exit $?
  bash scripts/gpu_ab_variant.sh ${TAG}_nt nt "" "" "c2 c3"
  exit $?
fi
if [ "$MODE" = dropin ]; then
  # the wdl drop-in fit (load-style train_epoch) at C5 shapes: its tests, then bench's dropin_fit
  timeout -k 10 300 python -u -m pytest tests/test_gpu_dropin.py tests/test_gpu_parity.py -m gpu -q -rf -k "wdl or load_style or running_loss" \
    -p no:cacheprovider --timeout 200 --timeout-method thread > $OUT/pytest_dropin.log 2>&1
  rc=$?; echo "pytest rc=$rc: $(tail -1 $OUT/pytest_dropin.log)"; [ $rc -eq 0 ] || { grep -E "^(FAILED|ERROR)" $OUT/pytest_dropin.log; exit $rc; }
  timeout -k 10 300 python -c "
import bench, json, argparse
a = argparse.Namespace(batch=65536)
print(json.dumps(bench.dropin_fit(a)))" > $OUT/dropin.json 2> $OUT/dropin.err || { tail -5 $OUT/dropin.err; exit 1; }
  cat $OUT/dropin.json
  exit 0
fi
if [ "$MODE" = nowait ]; then
  # probe: the compute stream's cross-stream wait on the prefetch replaced by a host wait
  for rep in 1 2; do
    for cfg in c5:0 c5:1 c2:0 c2:1; do
      IFS=: read wl e <<< "$cfg"
      DLAMD_PF_NOWAIT=$e timeout -k 10 300 python bench.py --no-cpu-baseline --no-extra --workload $wl \
        --steps 20 --warmup 5 > $OUT/nw_${wl}_$e.json 2> $OUT/nw_${wl}_$e.err || { tail -5 $OUT/nw_${wl}_$e.err; exit 1; }
      python -c "
import json;d=json.loads(open('$OUT/nw_${wl}_$e.json').read().strip().splitlines()[-1])
print('$wl pf_nowait=$e', d['ms_per_step'], 'host', d.get('host_submit_ms_per_step'))"
    done
  done
  DLAMD_PF_NOWAIT=1 bash scripts/gpu_r4.sh trace ${TAG}_nw c5
  exit $?
fi
if [ "$MODE" = check ]; then
  # the GPU suite without the full-size tests, then C2 / C5 benches and a C2 trace
  bash scripts/gpu_r4.sh quick $TAG || exit $?
  for wl in c2 c5; do
    timeout -k 10 300 python bench.py --no-cpu-baseline --no-extra --workload $wl --steps 20 --warmup 5 \
      > $OUT/b_$wl.json 2> $OUT/b_$wl.err || { tail -5 $OUT/b_$wl.err; exit 1; }
    python scripts/bench_brief.py $OUT/b_$wl.json
  done
  bash scripts/gpu_r4.sh trace $TAG c2
  exit $?
fi
if [ "$MODE" = status ]; then
  # the per-step status read-back (a D2H copy into pinned memory after every step) every 1 / 16 steps
  for rep in 1 2; do
    for cfg in c5:1 c5:16 c2:1 c2:16; do
      IFS=: read wl e <<< "$cfg"
      DLAMD_STATUS_EVERY=$e timeout -k 10 300 python bench.py --no-cpu-baseline --no-extra --workload $wl \
        --steps 20 --warmup 5 > $OUT/st_${wl}_$e.json 2> $OUT/st_${wl}_$e.err || { tail -5 $OUT/st_${wl}_$e.err; exit 1; }
      python -c "
import json;d=json.loads(open('$OUT/st_${wl}_$e.json').read().strip().splitlines()[-1])
print('$wl status_every=$e', d['ms_per_step'], 'host', d.get('host_submit_ms_per_step'))"
    done
  done
  DLAMD_STATUS_EVERY=16 bash scripts/gpu_r4.sh trace ${TAG}_s16 c5
  exit $?
fi
if [ "$MODE" = prio ]; then
  # stream priorities: side (index prefetch) / main (the step) — default -1 / 0
  for rep in 1 2; do
    for cfg in c5:-1:x c5:-1:-1 c5:0:x c2:-1:x c2:-1:-1; do
      IFS=: read wl sp mp <<< "$cfg"
      if [ $mp = x ]; then MP=""; else MP="DLAMD_MAIN_PRIORITY=$mp"; fi
      env DLAMD_SIDE_PRIORITY=$sp $MP timeout -k 10 300 python bench.py --no-cpu-baseline --no-extra --workload $wl \
        --steps 20 --warmup 5 > $OUT/pr_${wl}_${sp}_$mp.json 2> $OUT/pr_${wl}_${sp}_$mp.err || { tail -5 $OUT/pr_${wl}_${sp}_$mp.err; exit 1; }
      python -c "
import json;d=json.loads(open('$OUT/pr_${wl}_${sp}_$mp.json').read().strip().splitlines()[-1])
print('$wl side=$sp main=$mp', d['ms_per_step'], 'host', d.get('host_submit_ms_per_step'))"
    done
  done
  DLAMD_MAIN_PRIORITY=-1 bash scripts/gpu_r4.sh trace ${TAG}_mp c5
  exit $?
fi
if [ "$MODE" = pfeager ]; then
  # the prefetch's index build as a graph replay (0) or eager launches (1) on the side stream;
  # and no prefetch at all
  for rep in 1 2; do
    for cfg in c5:0 c5:1 c2:0 c2:1; do
      IFS=: read wl e <<< "$cfg"
      DLAMD_PF_EAGER=$e timeout -k 10 300 python bench.py --no-cpu-baseline --no-extra --workload $wl \
        --steps 20 --warmup 5 > $OUT/pe_${wl}_$e.json 2> $OUT/pe_${wl}_$e.err || { tail -5 $OUT/pe_${wl}_$e.err; exit 1; }
      python -c "
import json;d=json.loads(open('$OUT/pe_${wl}_$e.json').read().strip().splitlines()[-1])
print('$wl pf_eager=$e', d['ms_per_step'], 'host', d.get('host_submit_ms_per_step'))"
    done
    timeout -k 10 300 python bench.py --no-cpu-baseline --no-extra --workload c5 --no-prefetch --steps 20 --warmup 5 \
      > $OUT/pe_c5_nopf.json 2> $OUT/pe_c5_nopf.err || exit 1
    python -c "
import json;d=json.loads(open('$OUT/pe_c5_nopf.json').read().strip().splitlines()[-1])
print('c5 no prefetch', d['ms_per_step'], 'host', d.get('host_submit_ms_per_step'))"
  done
  DLAMD_PF_EAGER=1 bash scripts/gpu_r4.sh trace ${TAG}_e1 c5
  exit $?
fi
if [ "$MODE" = pfdepth ]; then
  # prefetch depth (batches in flight on the side stream) x submission order, then a C5 trace
  timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -rf -k prefetch -p no:cacheprovider \
    --timeout 120 --timeout-method thread > $OUT/pytest_pf.log 2>&1
  rc=$?; echo "pytest rc=$rc: $(tail -1 $OUT/pytest_pf.log)"; [ $rc -eq 0 ] || { grep -E "^(FAILED|ERROR)" $OUT/pytest_pf.log; exit $rc; }
  for rep in 1 2; do
    for cfg in c5:1:0 c5:2:0 c5:2:1 c2:1:0 c2:2:0; do
      IFS=: read wl d a <<< "$cfg"
      DLAMD_PF_DEPTH=$d DLAMD_PF_AFTER=$a timeout -k 10 300 python bench.py --no-cpu-baseline --no-extra --workload $wl \
        --steps 20 --warmup 5 > $OUT/pf_${wl}_${d}_${a}.json 2> $OUT/pf_${wl}_${d}_${a}.err || { tail -5 $OUT/pf_${wl}_${d}_${a}.err; exit 1; }
      python -c "
import json;d=json.loads(open('$OUT/pf_${wl}_${d}_${a}.json').read().strip().splitlines()[-1])
print('$wl depth=$d after=$a', d['ms_per_step'], 'host', d.get('host_submit_ms_per_step'))"
    done
  done
  DLAMD_PF_DEPTH=2 bash scripts/gpu_r4.sh trace ${TAG}_d2 c5
  exit $?
fi
if [ "$MODE" = pfab ]; then
  # the next batch's prefetch submitted before (0) or after (1) the step's own graph
  for wl in c5 c2; do
    for a in 0 1 0 1; do
      DLAMD_PF_AFTER=$a timeout -k 10 300 python bench.py --no-cpu-baseline --no-extra --workload $wl --steps 20 \
        --warmup 5 > $OUT/pf_${wl}_$a.json 2> $OUT/pf_${wl}_$a.err || { tail -5 $OUT/pf_${wl}_$a.err; exit 1; }
      python -c "
import json;d=json.loads(open('$OUT/pf_${wl}_$a.json').read().strip().splitlines()[-1])
print('$wl pf_after=$a', d['ms_per_step'], 'host', d.get('host_submit_ms_per_step'))"
    done
  done
  DLAMD_PF_AFTER=1 bash scripts/gpu_r4.sh trace ${TAG}_pf1 c5
  exit $?
fi
if [ "$MODE" = abdiag ]; then
  # the root Adam state against TF's v (libdlamd_vst), then the backward's byte split
  bash scripts/gpu_ab_variant.sh ${TAG}_vst vst "" "" "c2 c5" || exit $?
  bash scripts/gpu_r4.sh bwddiag $TAG
  exit $?
fi
if [ "$MODE" = bwddiag ]; then
  # the backward's excess line fetches split by access stream: C2 FETCH_SIZE / WRITE_SIZE passes
  # for the default build and the DL_BWD_DIAG builds (d1: dx0 slices, d2: fm_sum rows, d8: no
  # record writes — each redirected to a cache-resident address; wrong results, bytes only)
  for V in new d1 d2 d8; do
    W=$OUT/bwd_$V; mkdir -p $W
    if [ $V = new ]; then VV=""; else VV=$V; fi
    args="--no-cpu-baseline --no-extra --workload c2"
    DLAMD_VARIANT=$VV timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $W/prof_fetch -o fetch -- \
      python bench.py --steps 3 --warmup 1 $args > $W/prof_fetch.log 2>&1
    rc=$?; echo "$V fetch rc=$rc"; [ $rc -eq 0 ] || exit $rc
    DLAMD_VARIANT=$VV timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $W/prof_write -o write -- \
      python bench.py --steps 3 --warmup 1 $args > $W/prof_write.log 2>&1
    rc=$?; echo "$V write rc=$rc"; [ $rc -eq 0 ] || exit $rc
    python scripts/pmc_summary.py $W $W/pmc_summary.json c2 > $W/summary.txt && grep -i "bwd\|gather" $W/summary.txt | head -6
  done
  exit 0
fi
echo "usage: gpu_r4.sh quick|full|bench|trace|combo|bwddiag TAG [variant]"; exit 2
