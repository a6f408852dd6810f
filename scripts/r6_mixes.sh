set -o pipefail
mkdir -p gpurun_out/r6
for m in slo phase-ts 8mix; do
  timeout -k 10 420 python -u bench.py --mix $m --reps 3 --steps 20 --warmup 3 --no-cu-check --out gpurun_out/r6/s1_$m.json > gpurun_out/r6/s1_$m.log 2>&1 || exit $?
done
