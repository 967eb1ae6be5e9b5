cd $GRAFT_REPO_ROOT
timeout -k 10 300 python tools/layer_table.py --top 200 > gpurun_out/layers.txt 2>&1 && \
timeout -k 10 300 python tools/conv_bench.py > gpurun_out/convbench.txt 2>&1
echo EXIT $?
