timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_learner.py tests/test_gpu_train_step.py > gpurun_out/r04v2_t.log 2>&1; rc=$?; tail -3 gpurun_out/r04v2_t.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 scripts/learner_mb.py vh > gpurun_out/r04v2_mb.txt 2>&1; cat gpurun_out/r04v2_mb.txt
