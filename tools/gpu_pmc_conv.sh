# PMC passes over tools/conv_bench.py for the shapes in $SHAPES (one rocprofv3 run per pass)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export REPS=2
i=0
for pmc in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_WAIT_INST_LDS" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INSTS_VMEM_RD SQ_WAVES GRBM_GUI_ACTIVE" \
           "TCC_HIT TCC_MISS TCP_TCC_READ_REQ_sum GRBM_COUNT"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $pmc --output-format csv -d gpurun_out/pmc$i -o run -- python tools/conv_bench.py $SHAPES > gpurun_out/pmc$i.log 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/pmc$i.log; }
done
