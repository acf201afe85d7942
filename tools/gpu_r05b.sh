set -u
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread tests/test_solver_gpu.py::test_one_exact_step_high_rpc_degree tests/test_edge_cases.py::test_single_observation_points_and_frames tests/test_eval_forms_gpu.py > $OUT/pytest_r05b.log 2>&1; echo "pytest rc $?"
timeout -k 10 300 python -u tools/cg_form_probe.py > $OUT/cg_probe_r05b.log 2>&1 || exit 1
MVBA_CG_TIMING=1 timeout -k 10 300 python bench.py --shard-of 8 --steps 200 --ba-iters 3 --no-cpu-baseline --mesh-subdiv 0 > $OUT/s8_timing_r05b.log 2>&1 || exit 1
MVBA_CG_TIMING=1 timeout -k 10 300 python bench.py --steps 200 --ba-iters 5 --no-cpu-baseline --mesh-subdiv 0 > $OUT/c2_timing_r05b.log 2>&1 || exit 1
grep "cg timing" $OUT/s8_timing_r05b.log $OUT/c2_timing_r05b.log
