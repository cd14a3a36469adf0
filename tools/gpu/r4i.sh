# r4i: secondary BASELINE configs with the round-4 code (seq512 fused + 8 x 64, GPT-2, XL auto).
set -o pipefail
bash tools/gpu/configs.sh
