set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/host_profile.py --concurrent 8 --n 3 > gpurun_out/host_prof_c8.txt 2>&1
