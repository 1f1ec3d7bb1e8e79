import json, sys
d = json.loads(sys.stdin.read())
r = d.get("roofline") or {}
ph = d.get("phase_ms")
print(d["value"], d["ms_per_step"], r.get("achieved"), r.get("other_syrk"), [round(x, 1) for x in ph] if ph else None)
