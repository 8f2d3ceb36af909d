set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/asr_timing.py --batch 1,8,32 --reps 5 > gpurun_out/asr_batch.log 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d /tmp/ab -o run -- python3 -u tools/asr_timing.py --batch 32 --reps 3 > gpurun_out/asr_batch_prof.log 2>&1
python tools/summarize_profile.py /tmp/ab/run_results.db "whisper-tiny transcribe_many, 32 utterances" > gpurun_out/asr_batch.md
