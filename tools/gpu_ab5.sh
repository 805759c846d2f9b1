set -o pipefail
bash tools/gpu_ab_quick.sh ab5 default@SSPP_G1=2 default@SSPP_G1=4 default@SSPP_NT=128,SSPP_G1=4 default@SSPP_NT=128,SSPP_G1=8 default@SSPP_NT=256,SSPP_G1=8 default@SSPP_G1=4,SSPP_HULL=0 || exit 1
SSPP_ABLATE=64 bash tools/gpu_ab_quick.sh ab5a default || exit 1
