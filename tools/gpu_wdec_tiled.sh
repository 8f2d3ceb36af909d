# Whisper decoder in the tiled layout + auto K split: numerics, then large-v3 / tiny timing
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_engine_gpu.py -k "whisper" tests/test_kernels_gpu.py -m gpu > gpurun_out/wdt_pytest.log 2>&1 || exit 11
timeout -k 10 300 python -u tools/asr_timing.py --asr whisper-large-v3 --reps 5 > gpurun_out/wdt_large.log 2>&1 || exit 12
timeout -k 10 200 python -u tools/asr_timing.py --asr whisper-tiny --reps 5 > gpurun_out/wdt_tiny.log 2>&1 || exit 13
