set -o pipefail
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_handoff.py tests/test_gpu_so.py tests/test_gpu_robust.py -k "not multi_handle" > gpurun_out/g1_tests.log 2>&1 && echo TESTS_OK
SEQALIB_HIP_LIB=seqalib_amd/lib/ab/libr5ctl.so timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_gpu_handoff.py > gpurun_out/g1_control.log 2>&1; echo "control rc=$?"
