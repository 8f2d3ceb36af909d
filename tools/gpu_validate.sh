# GPU validation pass: every GPU test (one process), smoke, headline bench at the driver's 20/5
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/val_pytest.log 2>&1 || exit 11
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/val_smoke.log 2>&1 || exit 12
timeout -k 10 300 python -u bench.py > gpurun_out/val_bench.log 2>&1 || exit 13
