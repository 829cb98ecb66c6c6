set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-s6y}
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 || { tail -40 gpurun_out/${T}_pytest.log; exit 1; }
tail -1 gpurun_out/${T}_pytest.log
SHD_SEGSORT=bitonic timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "round or segments or zipf or device" > gpurun_out/${T}_pytest_bitonic.log 2>&1 || { tail -40 gpurun_out/${T}_pytest_bitonic.log; exit 1; }
tail -1 gpurun_out/${T}_pytest_bitonic.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
