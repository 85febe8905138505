#!/bin/bash
# round 5: time-to-k at C4a, three runs on one context (tools/r05_ttk_probe.py) with the Ritz
# trace, at the default 8 staging threads and at 16
set -u
for t in 8 16; do
  echo "threads=$t"; RBL_D2H_THREADS=$t RBL_RITZ_TRACE=1 timeout -k 10 200 python -u tools/r05_ttk_probe.py 2>&1 | tail -6 || exit 1
done
