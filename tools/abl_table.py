"""Print tools/ablate_wide.py JSON output as a kernel x library table (ms)."""
import json
import sys

t = open(sys.argv[1]).read()
d = json.loads(t[t.index("{"):])
libs = [k for k in d if isinstance(d[k], dict)]
names = list(d[libs[0]].keys())
print("kernel".ljust(14), *[l.split("/")[-1][:12].rjust(12) for l in libs])
for n in names:
    print(n.ljust(14), *[str(d[l][n]["ms"]).rjust(12) for l in libs])
