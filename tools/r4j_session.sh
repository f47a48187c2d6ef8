o=gpurun_out/r4j; mkdir -p $o
timeout -k 10 100 python -u tools/short_region.py --fresh 4 --reps 6 --idle-us 0 > $o/short_default.log 2>&1 || exit 1
FEDMI_SPIN_SYNC=1 timeout -k 10 100 python -u tools/short_region.py --fresh 4 --reps 6 --idle-us 0 > $o/short_spin.log 2>&1 || exit 1
for a in "1000 16" "8000 32"; do set -- $a; timeout -k 10 100 python -u tools/stamps.py $1 $2 50,200 bf16 emulate > $o/stamps_emulate_$1.log 2>&1 || exit 1; done
timeout -k 10 300 python -u -m pytest tests/test_hip_engine.py -m gpu -x -q -k "early_stop_fold_only or fused_eval" --timeout 120 --timeout-method thread > $o/pytest_es.log 2>&1; rc=$?; tail -3 $o/pytest_es.log; cat $o/short_*.log; exit $rc
