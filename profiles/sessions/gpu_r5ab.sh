# E-step stream count sweep (LDAEngine(streams=N), bench.py --streams): K = 100 shard, headline, 100 M events
mkdir -p gpurun_out/r5ab
for n in 4 5 6 3; do
  timeout -k 10 300 python -u bench.py --topics 100 --events 12500000 --steps 10 --warmup 3 --converge 0 --streams $n > gpurun_out/r5ab/k100_s$n.json 2> gpurun_out/r5ab/k100_s$n.err || exit 1
done
for n in 4 5; do
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --streams $n --e2e 0 --e2e-cold 0 > gpurun_out/r5ab/k20_s$n.json 2> gpurun_out/r5ab/k20_s$n.err || exit 1
done
for n in 4 5; do
  timeout -k 10 500 python -u bench.py --topics 100 --events 100000000 --steps 5 --warmup 2 --converge 0 --streams $n > gpurun_out/r5ab/k100m_s$n.json 2> gpurun_out/r5ab/k100m_s$n.err || exit 1
done
