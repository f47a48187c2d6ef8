o=gpurun_out/r4l; mkdir -p $o
timeout -k 10 200 python -u tools/probes/side_eval_probe.py > $o/side_eval.log 2>&1 || { cat $o/side_eval.log; exit 1; }
timeout -k 10 200 python -u tools/short_region.py --fresh 10 --fresh-only --shift-kb 0 0 0 4 64 1024 2048 0 4096 0 > $o/shift.log 2>&1
rc=$?; cat $o/side_eval.log $o/shift.log; exit $rc
