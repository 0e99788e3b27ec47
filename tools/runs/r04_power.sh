# GPU power and clock while the headline bench runs (is the int8 GEMM at the power cap?)
set -o pipefail
R=gpurun_out/r04_power
mkdir -p $R
cd "$GRAFT_REPO_ROOT"
(rocm-smi --showpower --showclocks --showmaxpower --json > $R/smi_idle.json 2>&1 || true)
timeout -k 10 200 python -u bench.py --steps 200 --warmup 3 --unpipelined-steps 100 --cpu-baseline 0 > $R/bench.json 2> $R/bench.err &
BP=$!
for i in $(seq 1 40); do
  sleep 0.5
  rocm-smi --showpower --showclocks --json >> $R/smi_samples.jsonl 2>/dev/null || true
  echo "" >> $R/smi_samples.jsonl
done
wait $BP
