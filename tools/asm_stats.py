"""Instruction histogram of one kernel in a hipcc -S device assembly file.
Usage: python tools/asm_stats.py file.s kernel_substring [--dump]"""
import re
import sys
from collections import Counter

path, key = sys.argv[1], sys.argv[2]
text = open(path).read()
start = None
for m in re.finditer(r'^(_Z\S+):', text, re.M):
    if key in m.group(1):
        start = m.start()
        name = m.group(1)
        break
if start is None:
    sys.exit("kernel not found")
end = text.find('.Lfunc_end', start)
body = text[start:end]
lines = [l.split(';')[0].strip() for l in body.split('\n')]
ins = [l for l in lines if l and not l.startswith(('.', '_')) and not l.endswith(':')]
c = Counter(l.split()[0] for l in ins)
print(name, len(ins), "instructions")
for k, v in c.most_common(70):
    print(f"  {k:36s}{v}")
if '--dump' in sys.argv:
    open('/tmp/kernel_dump.s', 'w').write(body)
