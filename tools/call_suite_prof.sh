set -o pipefail
bash tools/gpu_suite.sh && bash tools/profile_round.sh r3f
