set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
for v in -1 2 4 -1 2 4; do
  AVC_GEMM_BIGK=$v timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-wavenet --no-cpu-baseline --no-e2e --no-roofline --no-bf16 > gpurun_out/ab_$v.json 2>/dev/null || exit 1
  echo "$v $(python -c "import json;d=json.load(open('gpurun_out/ab_$v.json'));print(d['ms_per_step'])")" >> gpurun_out/ab.txt
done
