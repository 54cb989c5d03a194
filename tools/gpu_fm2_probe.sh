set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python3 tools/size_probe.py --sizes 65536,131072,196608,262144 --widths 2,4 --trees 6 --iters 40 > gpurun_out/fm2.json 2>gpurun_out/fm2.err || { tail -5 gpurun_out/fm2.err; exit 1; }
cat gpurun_out/fm2.json
