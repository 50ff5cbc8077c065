#!/bin/bash
# rocprofv3 kernel stats of the GPU speech features alone at B = 32 (the speech config) and B = 256.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for B in 32 256; do
  rm -rf gpurun_out/prof_audio_$B
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_audio_$B -o run -- \
    python3 tools/encoder_profile.py --enc audio --iters 5 --batch $B > gpurun_out/audio_$B.log 2>&1 || { echo "rc=$?"; tail -5 gpurun_out/audio_$B.log; exit 1; }
  python3 tools/prof_summary.py gpurun_out/prof_audio_$B/run_results.db --window spin --steps 5 > gpurun_out/audio_prof_$B.txt
  grep ms_per_iter gpurun_out/audio_$B.log; cut -c1-150 gpurun_out/audio_prof_$B.txt
done
