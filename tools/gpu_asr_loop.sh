# Whisper device-resident loop: tests, loop check, timing (tiny, large-v3)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_engine_gpu.py tests/test_e2e_gpu.py -k "whisper or asr or transcri" > gpurun_out/asrloop_pytest.log 2>&1 || exit 11
timeout -k 10 200 python -u tools/asr_loop_check.py > gpurun_out/asrloop_check.log 2>&1 || exit 12
timeout -k 10 200 python -u tools/asr_timing.py --asr whisper-tiny --reps 5 > gpurun_out/asrloop_tiny.log 2>&1 || exit 13
timeout -k 10 300 python -u tools/asr_timing.py --asr whisper-large-v3 --reps 3 > gpurun_out/asrloop_large.log 2>&1 || exit 14
