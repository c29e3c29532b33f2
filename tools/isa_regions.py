"""Static attribution of a kernel's instructions to source regions (round 5, VERDICT r4
"next" 2: attribute before cutting).  Disassembles one kernel of a code object built with
-gline-tables-only (`make -C simplepathtracer_amd/csrc gline`; same instructions as the
product build, checked by tools/isa_regions.py --compare), symbolizes every instruction
with its inline chain (llvm-symbolizer --inlining) and assigns it to the outermost phase
function on the chain:
  cast     find_closest (node walk + per-cast setup), test_leaf/test_group/ray_sphere
           (member tests: "members"), update_member ("update")
  sampler  coop_ball_vector (cube-minus-ball rejection sampler, RNG)
  shade    shade_step / refract_event / finish_step (rest of the shading step)
  refill   start_path* (primary ray + keyed RNG), take_items / claim_next, park/unpark
  loop     render_body's own code (ballots, refill rule, loop control, stats)
Prints static instruction counts (VALU, SALU, SMEM, VMEM, LDS, branch) per region.
Usage: python tools/isa_regions.py <code object> <kernel symbol> [--compare other.co]
"""
import collections
import re
import subprocess
import sys

LLVM = "/opt/rocm/lib/llvm/bin/"


def disasm(co, sym):
    out = subprocess.run([LLVM + "llvm-objdump", "-d", "--no-show-raw-insn", co], capture_output=True, text=True,
                         check=True).stdout
    lines, on = [], False
    for l in out.splitlines():
        if re.match(r"^[0-9a-f]+ <" + re.escape(sym) + ">:", l):
            on = True
            continue
        if on and not l.strip():
            break
        if on:
            m = re.match(r"\s+(\S+)(.*?)//\s*([0-9A-Fa-f]+):", l)
            if m:
                lines.append((int(m.group(3), 16), m.group(1), m.group(2).strip()))
    return lines


def kind(op):
    if op.startswith("v_"):
        return "valu"
    if op.startswith("s_load") or op.startswith("s_buffer_load") or op.startswith("s_dcache"):
        return "smem"
    if op.startswith("s_cbranch") or op.startswith("s_branch"):
        return "branch"
    if op.startswith("s_waitcnt") or op.startswith("s_nop") or op.startswith("s_sleep") or op.startswith("s_barrier"):
        return "wait"
    if op.startswith("s_"):
        return "salu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("global_", "buffer_", "flat_", "scratch_")):
        return "vmem"
    return "other"


PHASES = [  # (function-name fragment, region)
    ("update_member", "cast:update"),
    ("test_leaf", "cast:members"), ("test_group", "cast:members"), ("ray_sphere", "cast:members"),
    ("prim_list_cast", "cast:list"),
    ("find_closest", "cast:walk+setup"),
    ("coop_ball_vector", "sampler"),
    ("refract_event", "shade"), ("finish_step", "shade"), ("shade_step", "shade"),
    ("start_path", "refill"), ("claim_next", "refill"), ("park_path", "refill"), ("unpark_path", "refill"),
]


def region_of(chain):
    """chain: function names innermost first.  The innermost phase function decides (a
    uniform() draw inside coop_ball_vector is sampler; a normalize inside shade_step is
    shade; ray_sphere inside find_closest is cast:members)."""
    for n in chain:
        for frag, reg in PHASES:
            if frag in n:
                return reg
    return "loop"


def symbolize(co, addrs):
    inp = "\n".join(hex(a) for a in addrs)
    out = subprocess.run([LLVM + "llvm-symbolizer", "--obj=" + co, "--inlining", "--functions=short"], input=inp,
                         capture_output=True, text=True, check=True).stdout
    chains, cur = [], []
    blocks = out.strip("\n").split("\n\n")
    for b in blocks:
        ls = b.strip().splitlines()
        chains.append([ls[i] for i in range(0, len(ls), 2)])
    return chains


def main():
    co, sym = sys.argv[1], sys.argv[2]
    ins = disasm(co, sym)
    if "--compare" in sys.argv:
        other = disasm(sys.argv[sys.argv.index("--compare") + 1], sym)
        same = [a[1:] for a in ins] == [b[1:] for b in other]
        print(f"instruction streams identical: {same} ({len(ins)} vs {len(other)})")
    chains = symbolize(co, [a for a, _, _ in ins])
    tab = collections.defaultdict(collections.Counter)
    for (a, op, _), ch in zip(ins, chains):
        tab[region_of(ch)][kind(op)] += 1
    kinds = ["valu", "salu", "smem", "vmem", "lds", "branch", "wait", "other"]
    print(f"{'region':18s} " + " ".join(f"{k:>6s}" for k in kinds))
    for r in sorted(tab):
        print(f"{r:18s} " + " ".join(f"{tab[r][k]:6d}" for k in kinds))
    tot = collections.Counter()
    for r in tab:
        tot.update(tab[r])
    print(f"{'total':18s} " + " ".join(f"{tot[k]:6d}" for k in kinds))


if __name__ == "__main__":
    main()
