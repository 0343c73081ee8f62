"""Find the loops (backward branches) of one kernel in an llvm-objdump listing and count instruction classes in each
loop body (development tool).  usage: python tools/isa_loops.py <objdump.s> <kernel-name regex> [min body size]"""
import collections
import re
import sys

path, pat = sys.argv[1], sys.argv[2]
minsz = int(sys.argv[3]) if len(sys.argv) > 3 else 40
lines = open(path).read().split("\n")
start = None
for i, ln in enumerate(lines):
    if re.match(r"^[0-9a-f]+ <", ln):
        if start is not None:
            end = i
            break
        if re.search(pat, ln):
            start = i
else:
    end = len(lines)
ins = []  # (addr, mnemonic, text)
for ln in lines[start + 1:end]:
    m = re.search(r"//\s*([0-9A-F]+):", ln)
    t = ln.strip().split()
    if not m or not t:
        continue
    ins.append((int(m.group(1), 16), t[0], ln.strip()))
addr_idx = {a: k for k, (a, _, _) in enumerate(ins)}
print(lines[start][:120], "instructions:", len(ins))
for k, (a, mn, txt) in enumerate(ins):
    if not mn.startswith("s_cbranch") and mn != "s_branch":
        continue
    m = re.search(r"\+0x([0-9a-f]+)>", txt)
    if not m:
        continue
    base = ins[0][0] - 0  # offsets are relative to the symbol
    tgt = int(m.group(1), 16)
    # resolve target address: symbol start + offset
    sym0 = int(lines[start].split()[0], 16)
    ta = sym0 + tgt
    if ta > a or ta not in addr_idx:
        continue
    j = addr_idx[ta]
    body = ins[j:k + 1]
    if len(body) < minsz:
        continue
    c = collections.Counter()
    for _, m2, _ in body:
        if m2.startswith("v_") and "f64" in m2:
            c["valu_f64"] += 1
        elif m2.startswith("v_mad_u64") or m2.startswith("v_mul_hi") or m2.startswith("v_mul_lo") or m2.startswith("v_mad_"):
            c["valu_imul"] += 1
        elif m2.startswith("v_"):
            c["valu_other"] += 1
        elif m2.startswith("global_load") or m2.startswith("buffer_load"):
            c["vmem_ld"] += 1
        elif m2.startswith("global_store") or m2.startswith("buffer_store"):
            c["vmem_st"] += 1
        elif m2.startswith("ds_"):
            c["lds"] += 1
        elif m2.startswith("s_waitcnt"):
            c["waitcnt"] += 1
        elif m2.startswith("s_"):
            c["salu"] += 1
        else:
            c["other"] += 1
    print(f"loop {ins[j][0]:x}..{a:x}: {len(body)} instr", dict(c))
    if "-v" in sys.argv:
        oth = collections.Counter(m2 for _, m2, _ in body if m2.startswith("v_") and "f64" not in m2)
        print("   other VALU:", oth.most_common(25))
