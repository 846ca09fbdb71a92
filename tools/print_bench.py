import json,sys
d=json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
print(d["ms_per_step"], d["value"], d["parity"]["ok"] if d["parity"] else None, d["roofline"]["frac"])
print(json.dumps(d["real_envelope_detection"]))
print(json.dumps(d["draft_undecided"])[:700])
