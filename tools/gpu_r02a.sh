set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 500 --timeout-method thread > gpurun_out/pytest_gpu_r02a.log 2>&1
rc=$?
tail -30 gpurun_out/pytest_gpu_r02a.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py > gpurun_out/bench_r02a.log 2>&1
echo bench rc $?
tail -c 3000 gpurun_out/bench_r02a.log
