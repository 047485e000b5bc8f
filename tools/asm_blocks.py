"""Per-basic-block instruction census of a hipcc .s file (kernel tuning aid)."""
import re, sys, collections
blocks = collections.OrderedDict(); cur = "entry"
for ln in open(sys.argv[1]):
    m = re.match(r"^(\.?L\w+|\w+):", ln)
    if m:
        cur = m.group(1); blocks.setdefault(cur, collections.Counter()); continue
    m = re.match(r"^\s+([vs]_\w+|global_\w+|buffer_\w+|ds_\w+)", ln)
    if m:
        blocks.setdefault(cur, collections.Counter())[m.group(1)] += 1
for name, c in blocks.items():
    tot = sum(c.values()); valu = sum(v for k, v in c.items() if k.startswith("v_")); salu = sum(v for k, v in c.items() if k.startswith("s_"))
    if tot > 20:
        print(f"{name:28s} total={tot:4d} valu={valu:4d} salu={salu:4d}  top: " + ", ".join(f"{k}:{v}" for k, v in c.most_common(8)))
