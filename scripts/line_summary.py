"""One-line summary of a bench.py JSON line (the default line's headline and its riders)."""
import json
import sys

d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])


def one(tag, x):
    r = x.get("roofline") or {}
    dv = r.get("delivery") or {}
    c = x.get("cpu_baseline") or {}
    return (f"{tag} {x['value'] / 1e9:.3f} G ms {x['ms_per_step']:.4f} frac {r.get('frac') or 0:.4f} "
            f"k {r.get('kernel_ms_avg') or 0:.4f} traffic {r.get('traffic')} "
            + (f"dv frac {dv['frac']:.4f} span {dv['span_ms_avg']:.4f} " if dv else "")
            + (f"cpu {c.get('value', 0) / 1e6:.1f} M" if c else ""))


print(one("C3", d))
for k in ("at_1M_peers", "at_subcapacity", "at_epochs"):
    if k in d:
        print(one(k, d[k]))
