#!/bin/bash
# One GPU-box session: run the named steps in order and stop at the first failure.
#
#   gpurun --timeout 1200 -- bash scripts/gpu.sh tests bench prof
#
# steps:
#   tests     pytest -m gpu (PYTEST_FILES, default tests/; PYTEST_K: -k filter)
#   smoke     __graft_entry__.smoke()
#   bench     python bench.py $BENCH_ARGS                       -> $OUT/bench.json
#   prof      rocprofv3 --kernel-trace --stats of a short bench -> $OUT/prof_summary.md, timeline.txt
#   phases    scripts/bench_gs64.py --phases $PHASES_ARGS (per-bucket E-step times, phase cycles per chunk)
#   configs   scripts/bench_configs.sh (every BASELINE config on one GPU)
#   strong    scripts/strong_emulated.py (per-shard EM times for N = 2/4/8)
#   parity    scripts/precision_parity.py $PARITY_ARGS
#   micro     build + run scripts/micro/*.hip (fp64 latency / throughput probes)
#   pmc       rocprofv3 --pmc passes ($PMC = counter groups separated by ';', PMC_CMD = program, default a short bench)
#   cold      scripts/cold_start.py: where a cold ml_ops process spends its time
#   nccl      the one-rank RCCL test (tests/test_gpu_dist.py -k nccl)
#   ab        scripts/ab_env.sh $AB_ROUNDS $AB_VARIANTS (space-separated env settings, one per variant)
#   ranks     scripts/pipeline_ranks.py $RANKS_ARGS (per-rank stage seconds of the sharded ml_ops pipeline)
#   e2e       scripts/ab_e2e.sh $E2E_ROUNDS $E2E_VARIANTS (bench's ml_ops e2e wall under env variants)
# env: TAG (output dir gpurun_out/$TAG, default s), BENCH_ARGS, PROF_ARGS, PARITY_ARGS, PMC, PMC_ARGS, KEEP_GOING=1
# (this script replaces the per-experiment gpu_*.sh drivers of rounds 1-2; their records name them)
# (a failing pytest with exit status 1 -- assertion failures, not a crash -- does not stop the session)
set -u -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-s}
mkdir -p "$OUT"

stop() { echo "step $1 failed rc=$2"; exit "$2"; }

for s in "$@"; do
  echo "=== $s $(date +%T)"
  case $s in
    tests)
      timeout -k 10 1000 python -u -m pytest ${PYTEST_FILES:-tests} -m gpu -v --timeout 300 --timeout-method thread \
        ${PYTEST_K:+-k "$PYTEST_K"} > "$OUT/pytest_gpu.log" 2>&1
      rc=$?; grep -cE " PASSED" "$OUT/pytest_gpu.log"; grep -E "FAILED|ERROR" "$OUT/pytest_gpu.log" | head -20
      tail -2 "$OUT/pytest_gpu.log"
      if [ $rc -ne 0 ] && ! { [ $rc -eq 1 ] && [ "${KEEP_GOING:-0}" = 1 ]; }; then stop tests $rc; fi ;;
    smoke)
      timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || stop smoke $?
      tail -3 "$OUT/smoke.log" ;;
    bench)
      timeout -k 10 600 python -u bench.py ${BENCH_ARGS:-} > "$OUT/bench.log" 2>&1 || { tail -20 "$OUT/bench.log"; stop bench 1; }
      grep '^{' "$OUT/bench.log" | tail -1 > "$OUT/bench.json"; cut -c1-1500 "$OUT/bench.json" ;;
    prof)
      rm -rf "$OUT/prof"; mkdir -p "$OUT/prof"
      timeout -k 10 500 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run -- python3 bench.py \
        ${PROF_ARGS:---steps 10 --warmup 3 --converge 0 --e2e 0 --e2e-cold 0} > "$OUT/prof/bench.log" 2>&1 || { tail -20 "$OUT/prof/bench.log"; stop prof 1; }
      db=$(find "$OUT/prof" -name "*.db" | head -1)
      python scripts/prof_summary.py "$db" --top 30 --md "$OUT/prof_summary.md" > /dev/null
      python scripts/timeline.py "$db" --last-ms ${TIMELINE_MS:-6} > "$OUT/timeline.txt"
      rm -f "$db"; head -14 "$OUT/prof_summary.md" ;;
    phases)
      timeout -k 10 300 python -u scripts/bench_gs64.py --phases ${PHASES_ARGS:-} > "$OUT/phases.log" 2>&1 || { tail -20 "$OUT/phases.log"; stop phases 1; }
      grep '^{' "$OUT/phases.log" | cut -c1-600 ;;
    configs)
      OUTDIR="$OUT" timeout -k 10 1000 bash scripts/bench_configs.sh || stop configs $? ;;
    strong)
      timeout -k 10 1000 python -u scripts/strong_emulated.py ${STRONG_ARGS:-} --json "$OUT/strong.json" \
        --md "$OUT/strong.md" > "$OUT/strong.log" 2>&1 || { tail -20 "$OUT/strong.log"; stop strong 1; }
      cat "$OUT/strong.md" ;;
    parity)
      timeout -k 10 1100 python -u scripts/precision_parity.py ${PARITY_ARGS:-} --json "$OUT/parity.json" \
        --md "$OUT/parity.md" > "$OUT/parity.log" 2>&1 || { tail -20 "$OUT/parity.log"; stop parity 1; }
      cat "$OUT/parity.md" ;;
    micro)
      for f in scripts/micro/*.hip; do
        b=/tmp/$(basename "$f" .hip)
        hipcc --offload-arch=gfx950 -O3 "$f" -o "$b" || stop micro-build 1
        timeout -k 10 120 "$b" > "$OUT/$(basename "$f" .hip).txt" 2>&1 || stop micro $?
        cat "$OUT/$(basename "$f" .hip).txt"
      done ;;
    pmc)
      # PMC: counter groups separated by ';' (one rocprofv3 pass each); PMC_CMD: the profiled program
      i=0
      IFS=';' read -ra groups <<< "${PMC:?set PMC}"
      for g in "${groups[@]}"; do
        i=$((i + 1)); rm -rf "$OUT/pmc$i"; mkdir -p "$OUT/pmc$i"
        timeout -s KILL 120 rocprofv3 --pmc $g -d "$OUT/pmc$i" -o pmc -- python3 ${PMC_CMD:-bench.py ${PMC_ARGS:---steps 3 --warmup 1 --converge 0 --e2e 0 --e2e-cold 0}} \
          > "$OUT/pmc$i/log.txt" 2>&1 || stop pmc $?
        db=$(find "$OUT/pmc$i" -name "*.db" | head -1)
        python scripts/pmc_summary.py "$db" ${PMC_MATCH:+--match "$PMC_MATCH"} --md "$OUT/pmc_summary$i.md" > /dev/null
        rm -f "$db"; head -12 "$OUT/pmc_summary$i.md"
      done ;;
    cold)
      timeout -k 10 600 python -u scripts/cold_start.py ${COLD_ARGS:-} --md "$OUT/cold.md" --json "$OUT/cold.json" \
        > "$OUT/cold.log" 2>&1 || { tail -30 "$OUT/cold.log"; stop cold 1; }
      head -12 "$OUT/cold.md" ;;
    ab)
      timeout -k 10 1000 bash scripts/ab_env.sh ${AB_ROUNDS:-3} ${AB_VARIANTS:?set AB_VARIANTS} -- ${AB_ARGS:---steps 20 --warmup 5} \
        > "$OUT/ab.log" 2>&1 || { tail -20 "$OUT/ab.log"; stop ab 1; }
      cat "$OUT/ab.log" ;;
    ranks)
      timeout -k 10 1100 python -u scripts/pipeline_ranks.py ${RANKS_ARGS:-} --json "$OUT/ranks.json" \
        --md "$OUT/ranks.md" > "$OUT/ranks.log" 2>&1 || { tail -30 "$OUT/ranks.log"; stop ranks 1; }
      cat "$OUT/ranks.md" ;;
    e2e)
      timeout -k 10 1000 bash scripts/ab_e2e.sh ${E2E_ROUNDS:-2} ${E2E_VARIANTS:-ONI_PREFETCH=1} > "$OUT/ab_e2e.log" 2>&1 \
        || { tail -20 "$OUT/ab_e2e.log"; stop e2e 1; }
      cat "$OUT/ab_e2e.log" ;;
    nccl)
      timeout -k 10 300 python -u -m pytest tests/test_gpu_dist.py -m gpu -v -k nccl --timeout 120 \
        --timeout-method thread > "$OUT/nccl.log" 2>&1 || { tail -30 "$OUT/nccl.log"; stop nccl 1; }
      tail -3 "$OUT/nccl.log" ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
echo "=== done $(date +%T)"
