set -u
O=gpurun_out/r4l; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_spec_gpu.py tests/test_c4_gpu.py tests/test_templates_gpu.py tests/test_gpu_parity.py tests/test_gpu_abi.py > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -2 $O/t.log
timeout -k 10 200 python tools/host_enqueue.py 2147483648 1 > $O/he.log 2>&1 || { tail $O/he.log; exit 1; }
grep enqueue $O/he.log
STEPS=100 bash tools/ab.sh c4of8 libtfrg.so
