# RandomResizedCrop (LDS-banded) PMC: where does the 57 us go now? Two passes, each its own run.
source tools/gpu_job.sh
rm -rf gpurun_out/pmc_rrc_a gpurun_out/pmc_rrc_b
run 90 pmc_rrc_a timeout -s KILL 60 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS --kernel-trace -d gpurun_out/pmc_rrc_a -o k --output-format csv -- python3 tools/rrc_probe.py
run 90 pmc_rrc_b timeout -s KILL 60 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES SQ_BUSY_CYCLES FETCH_SIZE GRBM_GUI_ACTIVE --kernel-trace -d gpurun_out/pmc_rrc_b -o k --output-format csv -- python3 tools/rrc_probe.py
