set -u
TESTS="tests/test_bench_failure_gpu.py tests/test_solver_forms_gpu.py tests/test_cli.py" bash tools/gpu_r04.sh r04b tests || exit $?
bash tools/gpu_r04.sh r04b chol || exit $?
bash tools/gpu_r04.sh r04b pmc || exit $?
timeout -k 10 300 python bench.py > gpurun_out/bench_r04b.log 2>&1 || exit $?
python3 tools/bench_summary.py gpurun_out/bench_r04b.log
