# Round-4 session 9: every GPU test, then the headline and model benches, BERT trace, BERT knob A/B
set -o pipefail
bash tools/gpu_r4.sh tests bench bert wdb profb || exit 1
bash tools/gpu_r4.sh abbert
