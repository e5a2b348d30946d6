#!/bin/bash
# Summarise tools/gpu_call20.sh outputs (gpurun_out/).
tail -2 gpurun_out/gpu_tests.log
grep -h '^{' gpurun_out/probe_stripes.log gpurun_out/host_path.log
for f in b64_8192 b128_2048 b128_4096; do
  [ -f gpurun_out/$f.log ] && tail -1 gpurun_out/$f.log | python3 -c "
import json,sys;d=json.loads(sys.stdin.read());r=d['roofline'];o=d.get('roofline_other',{})
print('$f',d['value'],r.get('kernel'),r['frac'],o.get('kernel'),o.get('frac'))"
done
