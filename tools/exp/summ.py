#!/usr/bin/env python3
"""Summarise bench.py logs: value, encode / rebuild / parity-only us per launch, frac."""
import json
import sys

for f in sys.argv[1:]:
    try:
        d = json.loads([x for x in open(f) if x.startswith("{")][-1])
    except (IndexError, OSError, ValueError) as e:
        print(f, "no bench line", e)
        continue
    k = d["kernels"]
    print(f"{f}: value {d['value']} enc {k['encode']['avg_us']} dec {k['decode']['avg_us']} "
          f"frac {d['roofline']['frac']} dec_frac {d['roofline']['frac_decode']} "
          f"par {k['encode_parity_only']['avg_us']}/{k['encode_parity_only']['avg_us_back_to_back']} "
          f"verified {d['verified']}")
