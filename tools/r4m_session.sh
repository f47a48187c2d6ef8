o=gpurun_out/r4m; mkdir -p $o
export FEDMI_NO_BUILD=1
timeout -k 10 300 python -u -m pytest tests/test_hip_engine.py -m gpu -x -v -k "side_stream or lagged or early_stop_fold" --timeout 120 --timeout-method thread > $o/pytest_side.log 2>&1 || { tail -40 $o/pytest_side.log; exit 1; }
tail -3 $o/pytest_side.log
timeout -k 10 300 python -u tools/round_emulate.py --rows 1000 2000 4000 8000 --rounds 2000 --side ab --cases world1-fused lag+adamx+es rccl-lag+es > $o/emulate_side.log 2>&1 || { cat $o/emulate_side.log; exit 1; }
timeout -k 10 200 python -u tools/probes/side_eval_probe.py > $o/side_eval_probe.log 2>&1 || { cat $o/side_eval_probe.log; exit 1; }
grep "us/round" $o/emulate_side.log; cat $o/side_eval_probe.log
