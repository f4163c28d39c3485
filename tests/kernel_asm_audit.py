"""Hazard audit of the trunk kernels' inline-asm MFMA chains (forward_kernel.h mfma_split3).

The compiler pads hazards between the instructions it generates, but not into or out of an inline-asm
string, so the chains' correctness rests on what the compiler placed around them.  This audit reads
the gfx950 assembly of a translation unit (hipcc -S) and checks, per kernel that contains chains:

  1. no VALU instruction writes a chain's A/B operand or accumulator within the 2 wait states before
     the chain (VALU write -> MFMA operand);
  2. every other instruction touching a chain's accumulator is >= 20 wait states after the last
     chain that wrote it (MFMA D -> any reader or writer but the next MFMA taking it as C: 12 states
     for 8 passes, 19 for 16);
  3. inside every innermost loop (a backward branch) that runs chains, no other instruction touches
     the chains' accumulators (a copy the register allocator inserted); rule 1 also follows the
     loop's back-edge, so an operand written at the end of an iteration is checked against the
     chain that opens the next one.

Wait states are counted as issued instructions (s_nop N = N + 1).
"""
import re

REG = re.compile(r"\b([va])(?:\[(\d+):(\d+)\]|(\d+)\b)")
MEM_PREFIX = ("ds_", "global_", "buffer_", "scratch_", "flat_", "s_")


def regs_of(text):
    out = set()
    for m in REG.finditer(text):
        kind = m.group(1)
        if m.group(4) is not None:
            out.add((kind, int(m.group(4))))
        else:
            out.update((kind, r) for r in range(int(m.group(2)), int(m.group(3)) + 1))
    return out


class Inst:
    __slots__ = ("line", "op", "dst", "srcs", "all", "asm", "chain", "states", "label")

    def __init__(self, line, asm):
        self.line = line
        self.asm = asm
        self.chain = None
        self.label = None
        parts = line.split(None, 1)
        self.op = parts[0]
        ops = parts[1].split(";")[0] if len(parts) > 1 else ""
        fields = [f.strip() for f in ops.split(",")]
        self.dst = regs_of(fields[0]) if fields and fields[0] else set()
        self.srcs = regs_of(",".join(fields[1:]))
        self.all = self.dst | self.srcs
        m = re.match(r"s_nop\s+(\d+)", line)
        self.states = int(m.group(1)) + 1 if m else 1

    def is_valu_write(self):
        return self.op.startswith("v_") and not self.op.startswith("v_mfma") and not self.op.startswith(MEM_PREFIX)


def kernels(asm_text):
    """{kernel symbol: [Inst | ('label', name)]} for every function in an .s file."""
    lines = asm_text.split("\n")
    out = {}
    i = 0
    while i < len(lines):
        m = re.match(r"^(_Z\w+):", lines[i])
        if not m:
            i += 1
            continue
        name, body, in_asm = m.group(1), [], False
        i += 1
        while i < len(lines) and not lines[i].strip().startswith(".Lfunc_end"):
            t = lines[i].strip()
            i += 1
            if t.startswith(";;#ASMSTART"):
                in_asm = True
                continue
            if t.startswith(";;#ASMEND"):
                in_asm = False
                continue
            lm = re.match(r"^(\.LBB\w+):", t)
            if lm:
                body.append(("label", lm.group(1)))
                continue
            if not t or t.startswith((";", ".")) or t.endswith(":"):
                continue
            body.append(Inst(t, in_asm))
        out[name] = body
    return out


def audit_kernel(body):
    """Violations (strings) of rules 1-3 in one kernel's instruction list; [] when it has no chain."""
    insts = [x for x in body if isinstance(x, Inst)]
    # chains: maximal runs of consecutive asm instructions containing v_mfma
    chains = []
    cur = None
    for k, ins in enumerate(insts):
        if ins.asm and ins.op.startswith("v_mfma"):
            if cur is None:
                cur = {"first": k, "last": k, "D": set(), "AB": set()}
                chains.append(cur)
            cur["last"] = k
            cur["D"] |= ins.dst
            cur["AB"] |= ins.srcs - ins.dst
            ins.chain = cur
        elif not (ins.asm and ins.op.startswith("s_nop")):
            cur = None
    if not chains:
        return []
    bad = []
    allD = set().union(*(c["D"] for c in chains))
    # loops: backward branches; the innermost ones (no other loop inside) run the chains
    pos, idx = {}, 0
    for x in body:
        if isinstance(x, Inst):
            idx += 1
        else:
            pos[x[1]] = idx
    loops = []
    for k, ins in enumerate(insts):
        m = re.match(r"s_cbranch_\w+\s+(\.LBB\w+)|s_branch\s+(\.LBB\w+)", ins.line)
        if m:
            tgt = pos.get(m.group(1) or m.group(2))
            if tgt is not None and tgt <= k:
                loops.append((tgt, k))
    inner = [(a, b) for (a, b) in loops if not any((c, d) != (a, b) and a <= c and d <= b for (c, d) in loops)]
    top_of = {a: b for (a, b) in inner}    # loop top -> its back-edge branch

    # rule 1 (walking back across an innermost loop's back-edge too)
    def walk_back(k, need, c, seen):
        while k >= 0 and need > 0:
            ins = insts[k]
            if ins.chain is not None:
                return
            if ins.is_valu_write() and ins.dst & (c["AB"] | c["D"]):
                bad.append("rule 1: %r writes a chain operand %d states before it" % (ins.line, 2 - need))
            need -= ins.states
            if k in top_of and top_of[k] not in seen:
                seen.add(top_of[k])
                walk_back(top_of[k], need, c, seen)
            k -= 1
    for c in chains:
        k = c["first"]
        if k in top_of:      # the chain opens the loop: its predecessors are also the loop's tail
            walk_back(top_of[k], 2, c, {top_of[k]})
        walk_back(k - 1, 2, c, set())
    # rule 2
    for k, ins in enumerate(insts):
        if ins.chain is not None or not (ins.all & allD):
            continue
        states, j = 0, k - 1
        while j >= 0 and states < 20:
            if insts[j].chain is not None and insts[j].dst & ins.all:
                bad.append("rule 2: %r touches a chain accumulator %d states after the chain" % (ins.line, states))
                break
            states += insts[j].states
            j -= 1
    # rule 3: innermost loops running chains: nothing else touches their accumulators
    for (a, b) in inner:
        region = insts[a:b + 1]
        rc = [x.chain for x in region if x.chain is not None]
        if not rc:
            continue
        D = set().union(*(c["D"] for c in rc))
        for x in region:
            if x.chain is None and x.all & D:
                bad.append("rule 3: %r touches a chain accumulator inside the loop" % x.line)
    return bad


def audit(asm_text):
    """{kernel: (number of chains, violations)} for the kernels of an .s file that run chains."""
    out = {}
    for name, body in kernels(asm_text).items():
        insts = [x for x in body if isinstance(x, Inst)]
        n = sum(1 for x in insts if x.asm and x.op.startswith("v_mfma"))
        if n:
            out[name] = (n, audit_kernel(body))
    return out
