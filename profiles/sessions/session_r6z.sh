# (1) split segment sizes at K = 50 (1-day) and K = 100 (12.5 M shard), with the split's phase timer;
# (2) team4 GM at 3 waves per SIMD against the LDS-table team at 100 M events
set -u -o pipefail
cd /tmp && export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"; cd "$R"
O=$R/gpurun_out/r6z; mkdir -p $O
timeout -k 10 900 bash scripts/ab_env.sh 2 "ONI_GS_SPLIT_MIN=2048,words=96" "ONI_GS_SPLIT_MIN=2048,words=64" "ONI_GS_SPLIT_MIN=2048,words=48" "ONI_GS_SPLIT_MIN=2048,words=32" "ONI_GS_SPLIT_MIN=2048,words=24" -- --topics 50 --steps 20 --warmup 5 > $O/ab_split_k50.log 2>&1 || exit 1
cat $O/ab_split_k50.log
for w in 0 96 48; do
  if [ $w = 0 ]; then E="ONI_GS_SPLIT_MIN=2048"; else E="ONI_GS_SPLIT_MIN=2048,words=$w"; fi
  env $E timeout -k 10 300 python -u scripts/bench_gs64.py --phases --topics 50 > $O/phases_k50_w$w.log 2>&1 || exit 1
  echo "== K50 split words=$w"; grep '^{' $O/phases_k50_w$w.log | grep split | cut -c1-700
done
timeout -k 10 900 bash scripts/ab_env.sh 2 "ONI_GS_SPLIT_MIN=2048" "ONI_GS_SPLIT_MIN=2048,words=96" "ONI_GS_SPLIT_MIN=2048,words=64" -- --topics 100 --events 12500000 --steps 10 --warmup 3 > $O/ab_split_k100.log 2>&1 || exit 1
cat $O/ab_split_k100.log
for v in base gm3; do
  rm -rf /tmp/v_$v; cp -r "$R" /tmp/v_$v
  case $v in gm*) cp abvar/$v/_onihip*.so /tmp/v_$v/oni_ml_amd/_lib/ ;; esac
  (cd /tmp/v_$v && timeout -k 10 600 python -u scripts/bench_gs64.py --events 100000000 --topics 100 > $O/buckets_100m_$v.log 2>&1) || exit 1
  echo "== $v"; grep '^{' $O/buckets_100m_$v.log | grep -E 'team4|estep_graph' | cut -c1-160
  rm -rf /tmp/v_$v
done
