# targeted GPU tests (one pytest process)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu "$@" > gpurun_out/quick_pytest.log 2>&1 || exit 11
