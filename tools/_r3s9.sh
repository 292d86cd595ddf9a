mkdir -p gpurun_out/r3_step13
timeout -k 10 120 python -u tools/xattn_stamps.py > gpurun_out/r3_step13/stamps.log 2>&1 && bash tools/_r3s6.sh
rc=$?; cat gpurun_out/r3_step13/stamps.log; exit $rc
