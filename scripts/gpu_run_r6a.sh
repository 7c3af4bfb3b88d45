set -u
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r6a; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_memset.py tests/test_comm.py "tests/test_bench.py::test_bench_native_comm_leg_on_one_rank" tests/test_gpu_parity.py -k "memset or fill or comm or migrat or native or overlapped or Memcpy or memcpy or deadline or rank" > $O/pytest.log 2>&1; rc=$?; tail -5 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
PMC_PASSES="FETCH_SIZE;WRITE_SIZE;TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum;SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES;SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE" bash scripts/gpu_pmc_groups.sh r6a u8gather || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/f32trace -o run --output-format csv -- python3 tools/bench_configs.py --only f32lin --reps 10 > $O/f32lin.log 2>&1 || exit 1
grep '^{' $O/f32lin.log
echo done
