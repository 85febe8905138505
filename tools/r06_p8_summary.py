#!/usr/bin/env python3
"""Summarise a multi-rank bench line's per-rank record (round 6, tools/r06_p8_comm.sh)."""
import json
import sys

d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
pr = d.get("per_rank") or {}
print(f"value {d['value']} ms/run {d['ms_per_step']} transport {d['config']['transport']} "
      f"x{d['config']['transport_ranks']}  model {d.get('model')}")
for key in ("timed_ms_per_run", "stage_pass_ms_per_run", "stage_sum_ms", "unattributed_ms",
            "allreduce_host_us_per_call", "allreduce_dev_us_per_call", "exchange_host_us_per_call",
            "exchange_dev_us_per_call", "cpu_s_per_run", "allreduce_calls_per_run"):
    print(f"  {key:28s} {pr.get(key)}")
for s, v in (pr.get("stage_ms_per_run") or {}).items():
    print(f"  stage {s:22s} {v}")
print("  host_ms_per_run", pr.get("host_ms_per_run"))
print("  host_cpu", pr.get("host_cpu"))
print("  gpu_processes", pr.get("gpu_processes"))
