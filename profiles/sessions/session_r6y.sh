# (1) team4 at K = 100 with its chunk tables in the c.phi rows (GM) at 1 / 3 / 4 waves per SIMD, against the
#     LDS-table team (two workgroups per CU, LDS-bound); (2) the split plan's segment sizing at K = 50 and K = 100
set -u -o pipefail
cd /tmp && export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"; cd "$R"
O=$R/gpurun_out/r6y; mkdir -p $O
for v in base gm1 gm3 gm4 base2; do
  rm -rf /tmp/v_$v; cp -r "$R" /tmp/v_$v
  case $v in gm*) cp abvar/$v/_onihip*.so /tmp/v_$v/oni_ml_amd/_lib/ ;; esac
  (cd /tmp/v_$v && timeout -k 10 300 python -u scripts/bench_gs64.py --events 12500000 --topics 100 > $O/buckets_12m_$v.log 2>&1) || exit 1
  echo "== $v"; grep '^{' $O/buckets_12m_$v.log | grep -E 'team4|estep_graph' | cut -c1-140
  rm -rf /tmp/v_$v
done
timeout -k 10 900 bash scripts/ab_env.sh 3 "ONI_GS_SPLIT_MIN=2048" "ONI_GS_SPLIT_MIN=2048,words=128" "ONI_GS_SPLIT_MIN=2048,words=96" -- --topics 50 --steps 20 --warmup 5 > $O/ab_split_k50.log 2>&1 || exit 1
cat $O/ab_split_k50.log
timeout -k 10 900 bash scripts/ab_env.sh 2 "ONI_GS_SPLIT_MIN=2048" "ONI_GS_SPLIT_MIN=2048,words=128" -- --topics 100 --events 12500000 --steps 10 --warmup 3 > $O/ab_split_k100.log 2>&1 || exit 1
cat $O/ab_split_k100.log
