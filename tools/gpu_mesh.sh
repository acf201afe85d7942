set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_mesh.py tests/test_depth.py tests/test_tracks.py -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_mesh.log 2>&1
rc=$?; tail -30 gpurun_out/pytest_mesh.log; exit $rc
