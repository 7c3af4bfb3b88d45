#!/bin/bash
# Round-6 development run: focused GPU tests, UInt8 gather counters (LDS kernel), the UInt8
# register-window A/B, Float32 Linear kernel trace.  Output: gpurun_out/r6a/.
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r6a; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_memset.py tests/test_comm.py "tests/test_bench.py::test_bench_native_comm_leg_on_one_rank" tests/test_gpu_resample_fuzz.py tests/test_gpu_parity.py tests/test_gpu_slab_range.py "tests/test_gpu_large.py::test_zslab_linear_specials_in_halo_planes" > $O/pytest.log 2>&1; rc=$?; tail -5 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 tools/bench_configs.py --only u8win --reps 10 > $O/u8win.log 2>&1 || { tail $O/u8win.log; exit 1; }
grep '^{' $O/u8win.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/f32trace -o run --output-format csv -- python3 tools/bench_configs.py --only f32lin --reps 10 > $O/f32lin.log 2>&1 || exit 1
grep '^{' $O/f32lin.log
PMC_PASSES="FETCH_SIZE;WRITE_SIZE;TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum;SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES;SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE" bash scripts/gpu_pmc_groups.sh r6a u8gather || exit 1
echo done
