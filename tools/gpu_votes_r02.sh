set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python bench.py --no-cpu > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo "bench failed"; tail -30 gpurun_out/bench.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/bench.json'))
for k in ['value','ms_per_step','shard_of_8','p50_ms_4k_round','votes_device_2^20','e2e_votes_2^20','config2']: print(k, json.dumps(d.get(k))[:300])"
bash tools/gpu_pmc_votes.sh
