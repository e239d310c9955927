# C3 (fp32) and C5 (bf16 activations, one GPU) bench lines on the current tree (v5 temporal kernels)
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/c3c5
mkdir -p $OUT
timeout -k 10 400 python bench.py --config c3 --steps 3 --warmup 1 --no-cpu-baseline --no-roofline --no-alt-precision --launch eager > $OUT/c3.json 2> $OUT/c3.err || { tail -20 $OUT/c3.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/c3.json'));print('c3', d['ms_per_step'], d['value'], d.get('breakdown'))"
timeout -k 10 500 python bench.py --config c5 --steps 2 --warmup 1 --no-cpu-baseline --no-roofline --no-alt-precision --precision bf16 --launch eager > $OUT/c5.json 2> $OUT/c5.err || { tail -20 $OUT/c5.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/c5.json'));print('c5', d['ms_per_step'], d['value'], d.get('breakdown'))"
