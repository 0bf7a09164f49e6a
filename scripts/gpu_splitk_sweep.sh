# A/B of the split-K work-group target (TT2_SPLITK16_TARGET / TT2_SPLITK_TARGET) on the decoder + training legs
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
ARGS="--steps 2 --warmup 1 --no-cpu-baseline --no-wavenet --no-e2e --no-griffin-lim --train-steps 3"
for T in 512 256 1024 2048 512; do
  TT2_SPLITK16_TARGET=$T timeout -k 10 240 python bench.py $ARGS > gpurun_out/sk_$T.json 2> gpurun_out/sk_$T.err || { echo "fail $T"; tail -5 gpurun_out/sk_$T.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/sk_$T.json'));print('x3 target $T', d['value'], d['train']['ms_per_step'])"
done
for T in 256 1024; do
  TT2_SPLITK_TARGET=$T timeout -k 10 240 python bench.py $ARGS > gpurun_out/skf_$T.json 2> gpurun_out/skf_$T.err || { echo "fail $T"; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/skf_$T.json'));print('f32 target $T', d['value'], d['train']['ms_per_step'])"
done
