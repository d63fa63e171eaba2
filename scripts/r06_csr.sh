mkdir -p gpurun_out/r06/csr
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_oracle_scale.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -k "multi or MULTI or c4_multi or c5_multi or c3 or hub or inbound or mst or fused or c1" > gpurun_out/r06/csr/tests.log 2>&1
rc=$?; tail -3 gpurun_out/r06/csr/tests.log
if [ $rc -ne 0 ]; then grep -E "FAILED|Error|assert" gpurun_out/r06/csr/tests.log | head -20; exit $rc; fi
TAG=csrab LEGS=c4,c5 VARIANTS="GS_LIB_VARIANT=base;X=1;GS_LIB_VARIANT=base;X=1" scripts/r06_kstats.sh > /dev/null 2>&1
python3 scripts/r06_ab.py gpurun_out/r06/csrab
