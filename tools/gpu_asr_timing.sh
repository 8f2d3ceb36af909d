# Whisper transcription split (encoder / decoder per token), tiny and large-v3, + kernel trace of large-v3
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/asr_timing.py --asr whisper-tiny > gpurun_out/asr_tiny.log 2>&1 || exit 11
timeout -k 10 300 python -u tools/asr_timing.py --asr whisper-large-v3 --reps 5 > gpurun_out/asr_large.log 2>&1 || exit 12
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/asr_large_prof -o run -- python -u tools/asr_timing.py --asr whisper-large-v3 --reps 3 > gpurun_out/asr_large_prof.log 2>&1 || exit 13
