export TMPDIR=/tmp; mkdir -p gpurun_out/ab
timeout -k 10 600 python -u -m pytest -x -q --timeout 150 --timeout-method thread -m gpu tests > gpurun_out/ab/tests.log 2>&1; rc=$?; tail -3 gpurun_out/ab/tests.log; [ $rc = 0 ] || exit 1
bash tools/evidence_r04.sh 2
