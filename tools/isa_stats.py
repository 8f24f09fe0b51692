"""Instruction histogram per kernel of a hipcc -save-temps .s file (LDS / MFMA / VMEM forms, VGPRs).

python tools/isa_stats.py <file.s> <substring>...   e.g. gg_v3_kernelILi128ELi2ELi3ELi2ELi4E
"""
import collections
import re
import sys

src = open(sys.argv[1]).read()
for key in sys.argv[2:]:
    for m in re.finditer(r"^(_ZN5mxmoe\w*" + re.escape(key) + r"\w*):", src, flags=re.M):
        name = m.group(1)
        end = src.find(".Lfunc_end", m.end())
        body = src[m.end():end]
        c = collections.Counter(re.findall(r"^\s+((?:ds|buffer|global)_\w+|v_mfma\w*|s_waitcnt|s_barrier)", body, flags=re.M))
        meta = src[end:end + 4000]
        vg = re.search(r"; NumVgprs: (\d+)", meta)
        sc = re.search(r"; ScratchSize: (\d+)", meta)
        print(f"== {name[:90]}  vgprs={vg.group(1) if vg else '?'} scratch={sc.group(1) if sc else '?'}")
        for k, v in sorted(c.items()):
            print(f"   {v:6d} {k}")
