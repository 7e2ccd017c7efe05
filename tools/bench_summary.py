#!/usr/bin/env python3
"""One line per bench JSON file: window / steady q/s, ms/step, p50/p99, host enqueue, flagged blocks, kernel alone."""
import json
import sys


def load(path):
    for line in open(path):
        line = line.strip()
        if line.startswith("{") and '"metric"' in line:
            return json.loads(line)
    return None


for p in sys.argv[1:]:
    d = load(p)
    if not d:
        print(f"{p}: no bench line")
        continue
    if d.get("value") is None:
        print(f"{p}: ERROR {d.get('error')}")
        continue
    r = d["roofline"]
    st = d["steady_state"]
    he = d.get("host_enqueue_ms_per_step", {})
    ka = r.get("kernel_alone") or {}
    print(f"{p}: window {d['value']/1e3:.1f}k ({d['ms_per_step']*1e3:.1f} us) steady {st['value']/1e3:.1f}k "
          f"({st['ms_per_step']*1e3:.1f} us) p50 {d['p50_ms']:.3f} p99 {d['p99_ms']:.3f} "
          f"pipe {d['host_pipelined']['value']/1e3:.1f}k enq {he.get('window')}/{he.get('steady')} ms "
          f"frac {r['frac']} alone {ka.get('kernel_avg_us')}us/{ka.get('frac')} "
          f"flag {r['screen_fallbacks_timed']}/{r['screen_fallbacks_steady']} carry {r.get('carry_verify')}")
