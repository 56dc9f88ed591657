# Hardware counters of the team8 (longest documents) E-step kernel alone: one counter group per pass.
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/pmc8
i=0
for group in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_INSTS_VALU" "TCC_HIT_sum TCC_MISS_sum SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAIT_ANY SQ_INST_CYCLES_VMEM_RD" "TA_TA_BUSY_sum TA_FLAT_READ_WAVEFRONTS_sum TD_TD_BUSY_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum"; do
  i=$((i+1))
  rm -rf gpurun_out/pmc8/p$i
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $group -d gpurun_out/pmc8/p$i -o run -- python3 scripts/bench_gs64.py --only team8 --reps 2 --warm-em 2 > gpurun_out/pmc8/p$i.log 2>&1 || { echo "pass $i failed rc=$?"; tail -5 gpurun_out/pmc8/p$i.log; continue; }
  echo "pass $i ok"
done
for p in gpurun_out/pmc8/p*; do
  db=$(find $p -name "*.db" | head -1)
  [ -n "$db" ] && python scripts/pmc_summary.py "$db" --match gs_wsteam >> gpurun_out/pmc8/summary.md
done
cat gpurun_out/pmc8/summary.md
