set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out/r03p_core
bash tools/profile.sh r03p && python tools/summarize_prof.py gpurun_out/r03p > gpurun_out/r03p/summary.txt && cat gpurun_out/r03p/summary.txt && \
timeout -s KILL 60 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/r03p_core/pmc1 -o pmc -- tools/ubench/aes_core aesgh > gpurun_out/r03p_core/pmc1.log 2>&1 && \
timeout -s KILL 60 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT --output-format csv -d gpurun_out/r03p_core/pmc2 -o pmc -- tools/ubench/aes_core aesgh > gpurun_out/r03p_core/pmc2.log 2>&1 && \
python tools/summarize_prof.py gpurun_out/r03p_core > gpurun_out/r03p_core/summary.txt; cat gpurun_out/r03p_core/summary.txt; grep aesgh gpurun_out/r03p_core/pmc1.log
