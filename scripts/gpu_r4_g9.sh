set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4/g9_gpu_all.log 2>&1 &&
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4/g9_smoke.log 2>&1
