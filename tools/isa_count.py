"""Static instruction mix of one kernel in a hipcc -S listing.  usage: isa_count.py file.s symbol_prefix"""
import collections
import re
import sys

s = open(sys.argv[1]).read()
names = re.findall(r"^([A-Za-z0-9_]+):", s, re.M)
tgt = [n for n in names if n.startswith(sys.argv[2])]
n = tgt[0]
i = s.index(n + ":")
j = s.index(".Lfunc_end", i)
c = collections.Counter()
for line in s[i:j].splitlines():
    line = line.strip()
    if not line or line.startswith((".", ";")) or line.endswith(":"):
        continue
    c[line.split()[0]] += 1
print(n, "total static", sum(c.values()))
for k, v in c.most_common(int(sys.argv[3]) if len(sys.argv) > 3 else 40):
    print(f"  {k:28s}{v}")
