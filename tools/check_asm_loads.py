"""Guard for the inline-asm record loads of csrc/edge_lds.hip (the concat walk edge_lds_kernel and,
since round 6, the head-mean walk edge_lds_mean_kernel): compiles the file to gfx950 ISA and
follows each kernel's control flow (loop back edges included) for an instruction that reads or
writes a register an asm `global_load_dwordx2 ... s[..]` (scalar-base form, only the records use
it) may still be loading (those loads return in issue order; `s_waitcnt vmcnt(N)` retires one once
N of them were issued after it). The compiler treats the asm output as ready at once, so a copy or use it schedules
before the counted wait would read garbage.
    python tools/check_asm_loads.py [path/to/edge_lds.hip]   -> exit 1 on a finding"""
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "gat-pytorch_amd", "csrc", "edge_lds.hip")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")


def kernels(asm: str):
    name, body = None, []
    for line in asm.split("\n"):
        m = re.match(r"^(_Z\S*edge_lds(?:_mean)?_kernel\S*):", line)
        if m:
            name, body = m.group(1), []
            continue
        if name is not None:
            body.append(line)
            if "s_endpgm" in line:
                yield name, body
                name = None


def _insts(body):
    """(label or None, instruction text) in program order, comments and directives dropped;
    instructions from inline asm are tagged "asm:" (hipcc brackets them with ;;#ASMSTART/END)."""
    in_asm = False
    for line in body:
        raw = line.strip()
        if raw.startswith(";;#ASMSTART"):
            in_asm = True
            continue
        if raw.startswith(";;#ASMEND"):
            in_asm = False
            continue
        t = line.split(";")[0].strip()
        if not t or t.startswith("."):
            if re.match(r"^\.LBB\w+:", t):
                yield t[:-1], None
            continue
        yield None, ("asm:" + t) if in_asm else t


def _blocks(body):
    """Basic blocks: [(label, [instructions], successor labels)] split at labels and branches."""
    blocks, cur, label, n = [], [], "entry", 0
    for lab, t in _insts(body):
        if lab is not None:
            if cur or label == "entry":
                blocks.append([label, cur, None])
            label, cur = lab, []
            continue
        cur.append(t)
        if t.startswith(("s_branch", "s_cbranch", "s_endpgm", "s_setpc")):
            blocks.append([label, cur, None])
            n += 1
            label, cur = f"_fall{n}", []
    if cur:
        blocks.append([label, cur, None])
    for i, b in enumerate(blocks):
        last = b[1][-1] if b[1] else ""
        succ = []
        m = re.match(r"s_(c?)branch\S*\s+(\.LBB\w+)", last)
        if m:
            succ.append(m.group(2))
            if m.group(1) and i + 1 < len(blocks):
                succ.append(blocks[i + 1][0])
        elif not last.startswith("s_endpgm") and i + 1 < len(blocks):
            succ.append(blocks[i + 1][0])
        b[2] = succ
    return blocks


def _regs(op):
    for mm in re.finditer(r"v\[(\d+):(\d+)\]|\bv(\d+)\b", op):
        if mm.group(3):
            yield int(mm.group(3))
        else:
            yield from range(int(mm.group(1)), int(mm.group(2)) + 1)


_QMAX = 16   # tracked loads a path can have in flight


def _sgpr_pair(tok):
    m = re.fullmatch(r"s\[(\d+):(\d+)\]|(vcc|exec)", tok.strip())
    if not m:
        return None
    return m.group(3) if m.group(3) else f"s{m.group(1)}"


def _consts_after(consts, t):
    """Scalar flag values the compiler's structured control flow computes (the 64-bit masks it
    sets to 0 / -1 and tests through vcc), so branches those flags decide are followed only
    the way they go. Any other write to a tracked pair forgets it."""
    c = dict(consts)
    parts = t.split(None, 1)
    op = parts[0]
    ops = [o.strip() for o in parts[1].split(",")] if len(parts) > 1 else []
    dst = _sgpr_pair(ops[0]) if ops else None
    val = None
    if op == "s_mov_b64" and len(ops) == 2:
        if ops[1] in ("0", "-1"):
            val = int(ops[1])
        elif _sgpr_pair(ops[1]) in c:
            val = c[_sgpr_pair(ops[1])]
    elif op in ("s_xor_b64",) and len(ops) == 3 and ops[2] == "-1" and _sgpr_pair(ops[1]) in c:
        val = ~c[_sgpr_pair(ops[1])] & -1 if c[_sgpr_pair(ops[1])] == 0 else 0
        val = -1 if c[_sgpr_pair(ops[1])] == 0 else (0 if c[_sgpr_pair(ops[1])] == -1 else None)
    elif op == "s_andn2_b64" and len(ops) == 3 and ops[1] == "exec" and _sgpr_pair(ops[2]) in c:
        v = c[_sgpr_pair(ops[2])]
        val = 1 if v == 0 else (0 if v == -1 else None)     # exec assumed non-empty
    elif op == "s_and_b64" and len(ops) == 3 and ops[1] == "exec" and _sgpr_pair(ops[2]) in c:
        v = c[_sgpr_pair(ops[2])]
        val = 0 if v == 0 else (1 if v == -1 else None)
    if dst is not None:
        c.pop(dst, None)
        if val is not None:
            c[dst] = val
    if op.startswith(("s_cmp", "v_cmp")) or "vcc" in ops[:1]:
        if dst != "vcc":
            c.pop("vcc", None)
    return c


def _step(state, t, bad, where):
    """state: frozenset of (queue, consts); a queue is a tuple of (load site, (r0, r1)) in issue
    order (the newest last)."""
    out = set()
    for q, cst in state:
        consts = dict(cst)
        m = re.match(r"asm:global_load_dwordx2 v\[(\d+):(\d+)\], (v\d+), s\[", t)
        if m:
            regs = (int(m.group(1)), int(m.group(2)))
            if any(r in rr for _, rr in q for r in _regs(m.group(3))):
                bad.add((where, t))
            q = (tuple(x for x in q if not set(x[1]) & set(regs)) + ((where, regs),))[-_QMAX:]
            out.add((q, cst))
            continue
        # vmcnt(N) retires a tracked load once N tracked loads were issued after it: tracked
        # loads return in issue order, so with it pending so are they, and the count stays above
        # N whatever the compiler's own loads and stores do
        m = re.match(r"(?:asm:)?s_waitcnt vmcnt\((\d+)\)", t)
        if m:
            n = int(m.group(1))
            out.add((q[len(q) - n:] if n > 0 else (), cst))
            continue
        tt = t[4:] if t.startswith("asm:") else t
        if tt.startswith("s_"):
            out.add((q, frozenset(_consts_after(consts, tt).items())))
            continue
        parts = tt.split(None, 1)
        if q and len(parts) == 2:
            pend = {r for _, rr in q for r in rr}
            ops = [o.strip() for o in parts[1].split(",")]
            if any(r in pend for o in ops for r in _regs(o)):   # a read, or a write racing it
                bad.add((where, t))
        if parts[0].startswith("v_cmp") or "vcc" in tt:
            consts.pop("vcc", None)
        out.add((q, frozenset(consts.items())))
    return frozenset(out)


def _feasible(state, last):
    """The states that can take each edge of a block ending in `last`: (taken, fallthrough)."""
    m = re.match(r"s_cbranch_(vccnz|vccz)", last)
    if not m:
        return state, state
    taken, fall = set(), set()
    for q, cst in state:
        v = dict(cst).get("vcc")
        nz = None if v is None else (v != 0)
        want = m.group(1) == "vccnz"
        if nz is None or nz == want:
            taken.add((q, cst))
        if nz is None or nz != want:
            fall.add((q, cst))
    return frozenset(taken), frozenset(fall)


def scan(body):
    """Forward dataflow over the kernel's CFG to a fixed point: the possible in-flight load
    queues (with the scalar flags known on that path) at each block entry, union over
    predecessors, loop back edges included; load sites are static and queues bounded, so it
    terminates. Reports every instruction that reads or writes a register such a queue holds."""
    blocks = _blocks(body)
    index = {b[0]: k for k, b in enumerate(blocks)}
    entry = {b[0]: frozenset() for b in blocks}
    init = frozenset({((), frozenset())})
    if blocks:
        entry[blocks[0][0]] = init
    bad, work, seen = set(), ([blocks[0][0]] if blocks else []), set()
    while work:
        lab = work.pop()
        label, insts, succ = blocks[index[lab]]
        st = entry[lab] or init
        for k, t in enumerate(insts):
            st = _step(st, t, bad, f"{label}+{k}")
        last = insts[-1] if insts else ""
        last = last[4:] if last.startswith("asm:") else last
        taken, fall = _feasible(st, last)
        m = re.match(r"s_(c?)branch\S*\s+(\.LBB\w+)", last)
        for k2, s2 in enumerate(succ):
            if s2 not in index:
                continue
            part = taken if (m and k2 == 0) else fall
            if not part:
                continue
            new = entry[s2] | part
            if new != entry[s2] or s2 not in seen:
                entry[s2] = new
                seen.add(s2)
                work.append(s2)
    return sorted(bad)


def main():
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "k.s")
        subprocess.run([HIPCC, "-O3", "-std=c++17", "--offload-arch=gfx950", "--cuda-device-only",
                        "-S", "-o", out, SRC], check=True, capture_output=True)
        asm = open(out).read()
    found, n = 0, 0
    for name, body in kernels(asm):
        n += 1
        for where, t in scan(body):
            print(f"{name}: {where}: touches a register still loading: {t}")
            found += 1
    print(f"{n} kernels scanned, {found} findings")
    return 1 if found or n == 0 else 0


if __name__ == "__main__":
    sys.exit(main())
