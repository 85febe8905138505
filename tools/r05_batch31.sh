#!/bin/bash
# round 5, batch 31: the Ritz result in huge-page-advised memory (RBL_HOST_HUGEPAGE) — the
# time-to-k probe on both spectra and the bench's time-to-k records, alternating 0 / 1 on one box.
set -u
mkdir -p gpurun_out/r05_b31
export TMPDIR=/tmp
for hp in 0 1; do
  for spec in planted slow; do
    echo "== RBL_HOST_HUGEPAGE=$hp $spec" >> gpurun_out/r05_b31/ttk.log
    RBL_HOST_HUGEPAGE=$hp RBL_RITZ_TRACE=1 timeout -k 10 200 python -u tools/r05_ttk_probe.py $spec >> gpurun_out/r05_b31/ttk.log 2>&1 || { cat gpurun_out/r05_b31/ttk.log; exit 1; }
  done
done
cat gpurun_out/r05_b31/ttk.log | grep -v "^rbl_ritz"
for rep in 1 2; do
  for hp in 0 1; do
    RBL_HOST_HUGEPAGE=$hp timeout -k 10 300 python bench.py --steps 1 --warmup 1 --no-cpu-baseline --rmat-steps 0 --c3-steps 0 \
      > gpurun_out/r05_b31/ab_${hp}_$rep.json 2> gpurun_out/r05_b31/ab_${hp}_$rep.err || { tail -5 gpurun_out/r05_b31/ab_${hp}_$rep.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('gpurun_out/r05_b31/ab_${hp}_$rep.json').read().strip().splitlines()[-1])
t=d['time_to_k']; s=d['time_to_k_slow_spectrum']
print('hp=$hp', $rep, 'planted', t['seconds'], t['host_ms'], 'slow', s['seconds'], s['host_ms'])" | tee -a gpurun_out/r05_b31/ab.log
  done
done
