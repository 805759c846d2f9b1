set -o pipefail
bash tools/gpu_ab_quick.sh ab4 default w5 w6 default@SSPP_G1=4 default@SSPP_G1=16 || exit 1
EXTRA="--steps-per-launch 5" bash tools/gpu_ab_quick.sh ab4s default || exit 1
EXTRA="--steps-per-launch 10" bash tools/gpu_ab_quick.sh ab4s default || exit 1
