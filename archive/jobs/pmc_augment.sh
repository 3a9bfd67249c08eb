source tools/gpu_job.sh
run 300 pmc_rrc rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAVES --kernel-trace -d gpurun_out/pmc_rrc -o k --output-format csv -- python3 tools/rrc_probe.py
