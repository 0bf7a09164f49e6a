# PMC passes over the Postnet-only driver (conv_x3w_kernel): MFMA / LDS / wait counters, L2 hits
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4p
export TMPDIR=/tmp
timeout -k 10 120 python3 scripts/postnet_run.py 2 > gpurun_out/r4p/run.log 2>&1 || { tail -20 gpurun_out/r4p/run.log; exit 1; }
tail -2 gpurun_out/r4p/run.log
i=0
for pmc in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE" \
           "SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_MFMA SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM" \
           "TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum" "FETCH_SIZE"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $pmc -d gpurun_out/r4p/pmc$i -o run --output-format csv -- python3 scripts/postnet_run.py 2 > gpurun_out/r4p/pmc$i.log 2>&1 || { echo "pass $i rc=$?"; tail -5 gpurun_out/r4p/pmc$i.log; }
done
echo done
