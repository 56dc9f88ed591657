set -o pipefail
mkdir -p gpurun_out/sched
i=0
for spec in "default" "split|B8+B4|G64C+G64+G32|T1" "split|B8+B4+G32|G64C+G64|T1" "split+G32|B8+B4|G64C+G64|T1" "split|B8+B4|G64C+G64|T1+G32" "default" "split|B8+B4|G64C+G64+G32|T1" "split|B8+B4+G32|G64C+G64|T1"; do
  i=$((i+1))
  if [ "$spec" = default ]; then unset ONI_ESTEP_SCHED; else export ONI_ESTEP_SCHED="$spec"; fi
  timeout -k 10 200 python bench.py --steps 30 --warmup 3 --e2e 0 > gpurun_out/sched/$i.log 2>&1 || { echo "fail $spec"; tail -5 gpurun_out/sched/$i.log; exit 1; }
  echo "$spec $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/sched/$i.log)"
done
