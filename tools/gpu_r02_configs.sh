# round 2: kernel-configuration tables of the benchmark steps (tools/bench_conv_configs.py)
set -o pipefail
timeout -k 10 240 python -u tools/bench_conv_configs.py --out gpurun_out/r02_bench_conv_configs.txt > gpurun_out/cfg1.log 2>&1 || { tail -30 gpurun_out/cfg1.log; exit 1; }
timeout -k 10 240 python -u tools/bench_conv_configs.py --model attention_unet --batch 8 --out gpurun_out/r02_attention_conv_configs.txt > gpurun_out/cfg2.log 2>&1 || { tail -30 gpurun_out/cfg2.log; exit 1; }
timeout -k 10 240 python -u tools/bench_conv_configs.py --model multitask_unet --batch 8 --out gpurun_out/r02_multitask_conv_configs.txt > gpurun_out/cfg3.log 2>&1 || { tail -30 gpurun_out/cfg3.log; exit 1; }
timeout -k 10 300 python bench.py --cpu-baseline 0 > gpurun_out/bench_quick.json 2> gpurun_out/bench_quick.err || { tail -20 gpurun_out/bench_quick.err; exit 1; }
cat gpurun_out/r02_bench_conv_configs.txt
tail -1 gpurun_out/bench_quick.json
