# One GPU-box session, run on the box from the repo root:
#   bash tools/gpu_session.sh <tag> <stage>[,<stage>...]
# Stages (each step under its own time limit; the first failure ends the
# session, so nothing more runs on the GPU after a fault, abort or time-out):
#   probe    tools/stall_probe.py, 8-member groups with one-sample waves
#   hunt     the GPU suite HUNT_RUNS times with one-sample waves in group bands
#   tests    the GPU suite (per-test watchdog, tests/conftest.py)
#   smoke    __graft_entry__.smoke()
#   bench    the default bench line (python bench.py)
#   kt       rocprofv3 kernel traces of the bench (default command, --streams 1)
#   pmc      counter passes of the C3 trace kernel (tools/pmc_round.sh)
#   pmcall   counter passes C3 whole + 1/2, 1/4, 1/8 shares, C4, C5 (+ 1/8)
#   sb       one rank's share at N = 2/4/8 (four streams and one)
#   sbab     one rank's share, AB_VARIANTS alternated (SBAB_ROUNDS, SBAB_BANDS, SBAB_STREAMS, SBAB_STEPS)
#   cfg      C4 / C5 bench lines (whole frame and 1/8 share)
#   abx      interleaved A/B: AB_VARIANTS (default "base,default") on C3, C2, C4, C5 and C3 shares
#   e2e      rt_render end to end (RGBA8 and float)
#   e2etr    rt_render timelines: rocprofv3 runtime/marker/kernel/copy traces, tools/e2e_trace.py
#   wclk     per-wave clocks (needs lib/variants/wclk)
#   parity   full-size whole-frame oracle parity (tests -m fullsize)
# Output under gpurun_out/ (<stage>_<tag>.log); copy what is judged to profiles/.
set -o pipefail
tag=${1:?tag}
stages=${2:-tests,smoke,bench}
R=$GRAFT_REPO_ROOT
cd $R
export TMPDIR=/tmp
mkdir -p gpurun_out
out=gpurun_out
fail() { echo "$1-fail"; tail -${3:-30} "$2"; exit 1; }
has() { case ",$stages," in *",$1,"*) return 0;; esac; return 1; }

if has probe; then
  timeout -k 10 600 python -u tools/stall_probe.py --rounds ${PROBE_ROUNDS:-30} --sample-waves ${PROBE_SW:-1} \
    > $out/probe_$tag.log 2>&1 || fail probe $out/probe_$tag.log 60
  tail -1 $out/probe_$tag.log
fi
if has hunt; then
  # the whole suite, repeatedly, with one-sample waves in the group frames'
  # bands (the configuration of round 4's two stalled runs); a stall ends the
  # run through the per-test watchdog with the library's host-wait report
  for k in $(seq 1 ${HUNT_RUNS:-3}); do
    RT_TEST_GROUP_SAMPLE_WAVES=1 RT_TEST_WATCHDOG_S=60 timeout -k 10 400 python -u -m pytest tests -m gpu -x -v \
      --timeout 120 --timeout-method thread > $out/hunt${k}_$tag.log 2>&1 || fail hunt$k $out/hunt${k}_$tag.log 80
    tail -1 $out/hunt${k}_$tag.log
  done
fi
if has tests; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
    > $out/tests_$tag.log 2>&1 || fail tests $out/tests_$tag.log 60
  tail -1 $out/tests_$tag.log
fi
if has parity; then
  timeout -k 10 900 python -u -m pytest tests -m "gpu and fullsize" -x -v --timeout 170 --timeout-method thread \
    > $out/parity_$tag.log 2>&1 || fail parity $out/parity_$tag.log 60
  tail -1 $out/parity_$tag.log
fi
if has smoke; then
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke_$tag.log 2>&1 || fail smoke $out/smoke_$tag.log
  tail -1 $out/smoke_$tag.log
fi
if has bench; then
  timeout -k 10 300 python bench.py > $out/bench_$tag.log 2>&1 || fail bench $out/bench_$tag.log
  tail -1 $out/bench_$tag.log
fi
if has drv; then
  # the driver's own command (BENCH_rNN.json "cmd"), twice, its rocprofv3 kernel
  # trace (the timed window's fill / drain / per-frame spans: tools/kt_window.py),
  # and a 200-frame line for the window comparison
  for k in 1 2; do
    timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $out/drv${k}_$tag.log 2>&1 \
      || fail drv$k $out/drv${k}_$tag.log
    tail -1 $out/drv${k}_$tag.log | cut -c1-400
  done
  cd /tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$out/ktdrv_$tag -o run --output-format csv -- \
    python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $R/$out/ktdrv_$tag.log 2>&1 \
    || fail ktdrv $R/$out/ktdrv_$tag.log
  cd $R
  timeout -k 10 300 python3 bench.py --steps 200 --warmup 10 --no-cpu-baseline > $out/drv200_$tag.log 2>&1 \
    || fail drv200 $out/drv200_$tag.log
  tail -1 $out/drv200_$tag.log | cut -c1-400
fi
if has focus; then
  # the tests of what changed last (FOCUS: a pytest -k expression), before the whole suite
  timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "${FOCUS:?FOCUS}" \
    > $out/focus_$tag.log 2>&1 || fail focus $out/focus_$tag.log 40
  tail -1 $out/focus_$tag.log
fi
if has fetch; then
  # fetched bytes per frame of the timed path (the RT_FETCH_COUNT measuring build)
  timeout -k 10 300 python -u tools/fetch_bytes.py > $out/fetch_$tag.log 2>&1 || fail fetch $out/fetch_$tag.log
  cp profiles/canonical_counts.json $out/canonical_counts_$tag.json
  cat $out/fetch_$tag.log | cut -c1-300
fi
if has kt; then
  cd /tmp
  # the bench's timed frames (no moving camera: the in-flight instance's last 50 launches are the timed
  # frames; tools/kt_span.py --last 50 --with sky_batch_kernel gives their device time per frame, bench.py's
  # roofline.avg_kernel_ms)
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$out/kt_$tag -o run --output-format csv -- \
    python3 $R/bench.py --steps 50 --warmup 5 --no-cpu-baseline --moving-frames 0 > $R/$out/kt_$tag.log 2>&1 \
    || fail kt $R/$out/kt_$tag.log
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$out/kts1_$tag -o run --output-format csv -- \
    python3 $R/bench.py --steps 20 --warmup 3 --no-cpu-baseline --streams 1 --moving-frames 0 \
    > $R/$out/kts1_$tag.log 2>&1 || fail kts1 $R/$out/kts1_$tag.log
  cd $R
  echo kt-ok
fi
if has pmc; then
  bash tools/pmc_round.sh $tag > $out/pmcr_${tag}_C3_1.log 2>&1 || fail pmc $out/pmcr_${tag}_C3_1.log
  echo pmc-ok
fi
if has pmcall; then
  for cb in ${PMC_SET:-C3:1 C3:2 C3:4 C3:8 C4:1 C4:8 C5:1 C5:8}; do
    bash tools/pmc_round.sh $tag ${cb%%:*} ${cb##*:} > $out/pmcr_${tag}_${cb%%:*}_${cb##*:}.log 2>&1 \
      || fail pmc-$cb $out/pmcr_${tag}_${cb%%:*}_${cb##*:}.log
    echo pmc-ok-$cb
  done
fi
if has sb; then
  for n in 2 4 8; do
    timeout -k 10 300 python bench.py --steps 200 --warmup 5 --no-cpu-baseline --sim-bands $n \
      > $out/sb${n}_$tag.log 2>&1 || fail sb$n $out/sb${n}_$tag.log
    timeout -k 10 300 python bench.py --steps 50 --warmup 5 --no-cpu-baseline --sim-bands $n --streams 1 \
      > $out/sb${n}s1_$tag.log 2>&1 || fail sb${n}s1 $out/sb${n}s1_$tag.log
  done
  echo sb-ok
fi
if has sbab; then
  # one rank's share, library variants alternated (AB_VARIANTS; bench.py --lib)
  for r in $(seq ${SBAB_ROUNDS:-2}); do
    for v in ${AB_VARIANTS//,/ }; do
      lib=""
      [ "$v" != default ] && lib="--lib $v"
      for n in ${SBAB_BANDS:-2 4 8}; do
        for s in ${SBAB_STREAMS:-4 1}; do
          f=$out/sbab_${tag}_${v}_${n}_${s}_$r.log
          timeout -k 10 300 python bench.py --steps ${SBAB_STEPS:-200} --warmup 5 --no-cpu-baseline --sim-bands $n \
            --streams $s $lib > $f 2>&1 || fail sbab-$v-$n-$s $f
          grep '^{' $f | tail -1 | python3 -c "import sys, json; d = json.loads(sys.stdin.read()); \
print(json.dumps({'variant': '$v', 'bands': $n, 'streams': $s, 'round': $r, 'ms_per_step': round(d['ms_per_step'], 5), \
'kernel_ms': round(d['config']['kernel_ms_per_frame'], 5), 'launch': d['config'].get('timed_launch')}))" \
            >> $out/sbab_$tag.jsonl
        done
      done
    done
  done
  cat $out/sbab_$tag.jsonl
fi
if has lines; then
  # bench lines alternated over LINES_ROUNDS rounds: LINES="args a|args b|..." (each a bench.py argument set,
  # --no-cpu-baseline --moving-frames 0 added); one summary JSON line per run into lines_<tag>.jsonl
  IFS='|' read -ra sets <<< "${LINES:?LINES}"
  for r in $(seq ${LINES_ROUNDS:-2}); do
    for i in "${!sets[@]}"; do
      a="${sets[$i]}"
      f=$out/lines_${tag}_${i}_$r.log
      timeout -k 10 300 python bench.py --no-cpu-baseline --moving-frames 0 $a > $f 2>&1 || fail lines-$i $f
      grep '^{' $f | tail -1 | LARGS="$a" R=$r python3 -c "import sys, json, os; d = json.loads(sys.stdin.read()); \
c = d['config']; print(json.dumps({'args': os.environ['LARGS'], 'round': int(os.environ['R']), 'mrays': round(d['value'], 1), \
'ms_per_step': round(d['ms_per_step'], 5), 'kernel_ms': round(c['kernel_ms_per_frame'], 5), \
'lone_kernel_ms': round(c['lone_kernel_ms_per_frame'], 5), 'launch': c.get('timed_launch')}))" >> $out/lines_$tag.jsonl
    done
  done
  cat $out/lines_$tag.jsonl | cut -c1-300
fi
if has cfg; then
  for c in C2 C4 C5; do
    timeout -k 10 300 python bench.py --config $c --steps 5 --warmup 1 --no-cpu-baseline --moving-frames 0 \
      > $out/bench_${c}_$tag.log 2>&1 || fail bench-$c $out/bench_${c}_$tag.log
  done
  for c in C4 C5; do
    timeout -k 10 300 python bench.py --config $c --steps 5 --warmup 1 --no-cpu-baseline --moving-frames 0 --sim-bands 8 \
      > $out/sb8_${c}_$tag.log 2>&1 || fail sb8-$c $out/sb8_${c}_$tag.log
  done
  echo cfg-ok
fi
if has abx; then
  for c in ${ABX_CONFIGS:-C3 C2 C4 C5}; do
    timeout -k 10 300 python tools/abx.py --config $c --variants ${AB_VARIANTS:-base,default} --rounds ${ABX_ROUNDS:-6} \
      --frames 8 >> $out/abx_$tag.log 2>&1 || fail abx-$c $out/abx_$tag.log
  done
  for b in ${ABX_BANDS:-0/8 0/4 0/2}; do
    timeout -k 10 300 python tools/abx.py --config C3 --band $b --variants ${AB_VARIANTS:-base,default} \
      --rounds ${ABX_ROUNDS:-6} --frames 12 >> $out/abx_$tag.log 2>&1 || fail abx-$b $out/abx_$tag.log
  done
  grep variant $out/abx_$tag.log
fi
if has e2e; then
  for fl in 8 0; do
    timeout -k 10 200 python tools/e2e_probe.py --config C3 --frames 12 --flags $fl >> $out/e2e_$tag.log 2>&1 \
      || fail e2e $out/e2e_$tag.log
  done
  echo e2e-ok
fi
if has e2etr; then
  # rt_render timelines (runtime + marker + kernel + copy traces; no counters)
  cd /tmp
  for fl in 8 0; do
    timeout -k 10 200 rocprofv3 --runtime-trace --marker-trace --kernel-trace --memory-copy-trace --output-format csv \
      -d $R/$out/e2etr_${fl}_$tag -o run -- python3 $R/tools/e2e_trace.py run --flags $fl --frames 12 \
      > $R/$out/e2etr_${fl}_$tag.log 2>&1 || fail e2etr-$fl $R/$out/e2etr_${fl}_$tag.log
  done
  cd $R
  for fl in 8 0; do python3 tools/e2e_trace.py analyse $out/e2etr_${fl}_$tag --flags $fl; done > $out/e2etr_$tag.jsonl \
    || fail e2etr-analyse $out/e2etr_$tag.jsonl
  echo e2etr-ok
fi
if has wclk; then
  timeout -k 10 300 python tools/wave_clock.py --config C3 --bands 1,2,4,8 > $out/wclk_$tag.log 2>&1 \
    || fail wclk $out/wclk_$tag.log
  echo wclk-ok
fi
echo ALLDONE
