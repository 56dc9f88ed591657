set -o pipefail
export KEEP_GOING=1
TAG=r3m_ph20 bash scripts/gpu.sh phases &&
timeout -k 10 600 bash scripts/ab_env.sh 3 "ONI_GS_XCD_SKIP=0" "ONI_GS_XCD_SKIP=1" -- --steps 20 --warmup 5 > gpurun_out/r3m_ab_xcd.log 2>&1 && grep ms_per_step gpurun_out/r3m_ab_xcd.log
