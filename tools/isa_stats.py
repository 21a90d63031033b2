"""Per-kernel ISA statistics of a gfx950 assembly file (hipcc --save-temps=obj):
global loads (and how many use SGPR-base addressing), VALU count, VGPRs, scratch."""
import re
import sys

s = open(sys.argv[1]).read()
labels = [(m.start(), m.group(1)) for m in re.finditer(r'^(_Z\w+):', s, re.M)]
for n, (pos, name) in enumerate(labels):
    end = labels[n + 1][0] if n + 1 < len(labels) else len(s)
    body = s[pos:end]
    short = re.search(r'k_[a-z0-9_]+', name)
    gl = len(re.findall(r'^\s+global_load', body, re.M))
    sad = len(re.findall(r'^\s+global_load\S* v\S+, v\d+, s\[', body, re.M))
    va = len(re.findall(r'^\s+v_', body, re.M))
    nv = re.search(r'NumVgprs:\s+(\d+)', body)
    sc = re.search(r'ScratchSize:\s+(\d+)', body)
    print(f"{short.group(0) if short else name:22s} gload={gl:4d} saddr={sad:4d} valu={va:5d} "
          f"vgpr={nv.group(1) if nv else '?':>4s} scratch={sc.group(1) if sc else '?'}")
