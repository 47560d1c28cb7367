set -u
O=gpurun_out/r4l; mkdir -p $O
for L in libtfrg.so libtfrg_np2.so; do
  for cfg in "2147483648 1" "494300000 2"; do
    echo "== $L $cfg"
    TFRG_LIB=$PWD/tfrecords-reader_amd/tfr_reader/$L timeout -k 10 200 python tools/host_enqueue.py $cfg > $O/he.log 2>&1 || { tail $O/he.log; exit 1; }
    grep -E "enqueue" $O/he.log
  done
done
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_spec_gpu.py tests/test_c4_gpu.py tests/test_templates_gpu.py tests/test_gpu_parity.py tests/test_gpu_abi.py > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -3 $O/t.log
