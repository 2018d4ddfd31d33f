cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/pmc5
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM SQ_INSTS_LDS -d gpurun_out/pmc5/sq -o run --output-format csv -- python3 tools/ab_bf3.py 2000000 2048 kernel=5 > gpurun_out/pmc5/sq.log 2>&1 || exit $?
timeout -s KILL 200 rocprofv3 --pmc TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum -d gpurun_out/pmc5/tc -o run --output-format csv -- python3 tools/ab_bf3.py 2000000 2048 kernel=5 > gpurun_out/pmc5/tc.log 2>&1 || exit $?
python3 tools/pmc_summary.py gpurun_out/pmc5
