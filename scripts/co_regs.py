"""Register / scratch / LDS use of kernels in an unbundled gfx950 code object (no GPU needed).

Usage: python scripts/co_regs.py DIR substr [substr ...]
DIR holds notes.txt (llvm-readelf --notes of the code object) and dis.txt (llvm-objdump -d of it);
prints, per kernel whose mangled name contains one of the substrings: VGPRs, SGPRs, private segment
(spill) bytes, LDS bytes, and how many scratch instructions sit within 60 instructions of an MFMA
(i.e. inside a streaming loop). Build the two files with:
  llvm-objcopy --dump-section=.hip_fatbin=fatbin.bin lib/obj/tci_rrlu.o
  clang-offload-bundler --type=o --input=fatbin.bin --targets=hipv4-amdgcn-amd-amdhsa--gfx950 --output=rrlu.co --unbundle
  llvm-readelf --notes rrlu.co > notes.txt; llvm-objdump -d --no-show-raw-insn rrlu.co > dis.txt
"""
import re
import sys

d, subs = sys.argv[1], sys.argv[2:]
notes = open(f"{d}/notes.txt").read()
meta = {}
for blk in notes.split("  - .agpr_count:")[1:]:
    name = re.search(r"\.name:\s+(\S+)", blk).group(1)
    g = lambda k: (re.search(r"\." + k + r":\s+(\d+)", blk) or [None, "?"])[1]  # noqa: E731
    meta[name] = (g("vgpr_count"), g("sgpr_count"), g("private_segment_fixed_size"), g("group_segment_fixed_size"))
funcs, cur = {}, None
for line in open(f"{d}/dis.txt").read().split("\n"):
    m = re.match(r"^[0-9a-f]+ <(.*)>:", line)
    if m:
        cur = m.group(1)
        funcs[cur] = []
    elif cur:
        funcs[cur].append(line)
for name, (v, s, p, lds) in meta.items():
    if not any(x in name for x in subs):
        continue
    body = funcs.get(name, [])
    sc = [i for i, l in enumerate(body) if "scratch_" in l]
    mf = [i for i, l in enumerate(body) if "v_mfma" in l]
    near = sum(1 for i in sc if any(abs(i - j) < 60 for j in mf))
    print(f"{name[:60]:60s} vgpr {v} sgpr {s} priv {p} lds {lds} | insts {len(body)} scratch {len(sc)} near-mfma {near}")
