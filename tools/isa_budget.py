"""Static VALU budget of a render_kernel instantiation, by loop phase and by
operation, from the kernel's gfx950 assembly with line tables.

    hipcc <Makefile flags> -gline-tables-only --cuda-device-only -S -o smallpt_g.s csrc/smallpt.hip
    python tools/isa_budget.py smallpt_g.s render_kernelILb0ELb0ELi0ELb1ELb0E

Each instruction is attributed twice through its `.loc` inlining chain:
  phase -- the outermost frame inside render_kernel's main loop: query (the
           sphere loop), pass B (bounce / camera ray), hit (shading of the
           hit), pass A (light sample / refraction), done (running average),
           prologue / epilogue (outside the loop);
  op    -- the innermost frame that is one of the costed operations: RNG
           draw, sphere test (query_bf / query2_bf body), sqrt_nr / rsq,
           rcp_nr, exact sqrt fallback, inv_len (vnorm), sincosf, powf
           (toInt), other.
Counts are static (instructions in the code, each executed once per pass of
its block); DESIGN.md §3 turns them into a per-iteration budget.
"""
import collections
import re
import sys

# smallpt.hip line ranges of render_kernel's loop phases (kept in step with the source)
SRC = "smallpt.hip"


def ranges(path):
    """Line ranges of the phases and ops, found by markers in the source."""
    src = open(path).read().split("\n")

    def find(pat, start=0):
        for i in range(start, len(src)):
            if re.search(pat, src[i]):
                return i + 1
        raise SystemExit("marker not found: %s" % pat)
    loop = find(r"^\s+while \(true\) \{\s*$", find(r"^render_kernel\("))
    pb = find(r"// ---- pass B", loop)
    q0 = find(r"if \(k >= nsamples\) \{", pb)
    hit = find(r"float dp = 0.f, inv_sign = 1.f;", q0)
    pa = find(r"// ---- pass A", hit)
    done = find(r"if \(done\) \{", pa)
    end = find(r"if \(GSTORE\) \{", done)
    multi = find(r"if \(a_L\) pass_a\(false\);", pa)
    phases = [("pass B", pb, q0), ("query", q0, hit), ("hit", hit, pa), ("pass A (>1 light)", multi, multi + 1),
              ("pass A", pa, done), ("done", done, end)]
    ops = [("RNG draw", find(r"float get_random_f\("), find(r"float get_random\(") + 3),
           ("sphere test (exact fallback)", find(r"float sphere_hit\("), find(r"int query_bf\(const G") - 1),
           ("sphere test", find(r"int query_bf\(const G"), find(r"^// ---------------------------------------------------------------------------", find(r"void query2_bf\("))),
           ("vnorm/inv_len", find(r"v3 vnorm\("), find(r"v3 vnorm\(")),
           ("toInt", find(r"int to_int\(float x\)"), find(r"int to_int\(float x\)") + 4)]
    return (loop, end), phases, ops


def main():
    asm, kern = sys.argv[1], sys.argv[2]
    srcdir = sys.argv[3] if len(sys.argv) > 3 else "se-195-project-ray-tracer_amd/csrc"
    (lstart, lend), phases, ops = ranges(srcdir + "/" + SRC)
    lines = open(asm).read().split("\n")
    start = next(i for i, l in enumerate(lines) if re.match(r"^\w*%s\w*:" % re.escape(kern), l))
    end = next(i for i in range(start, len(lines)) if lines[i].startswith(".Lfunc_end"))
    chain = []
    tab = collections.Counter()
    tot = collections.Counter()
    for l in lines[start:end]:
        s = l.strip()
        if s.startswith(".loc"):
            frames = re.findall(r"([\w./]+):(\d+):\d+", s.split(";", 1)[1] if ";" in s else "")
            chain = [(f.split("/")[-1], int(n)) for f, n in frames]      # innermost first
            continue
        if not s or s.startswith(".") or s.startswith(";") or s.endswith(":"):
            continue
        op = s.split()[0]
        if not op.startswith("v_"):
            continue
        phase = "prologue/epilogue"
        for f, n in reversed(chain):                                      # outermost first
            if f == SRC and lstart <= n < lend:
                phase = next((p for p, a, b in phases if a <= n < b), "loop control")
                break
        kind = "other"
        for f, n in chain:                                                # innermost first
            if f == "rt_glibc_math.h":
                if n <= 40:                      # (bit-cast / fma helpers: the caller decides)
                    continue
                kind = "sincosf" if n >= 183 else "powf (toInt)"
                break
            if f == "rt_common.h":
                kind = {True: "sqrt_nr / rsq"}.get(True)
                src = open(srcdir + "/rt_common.h").read().split("\n")
                fn = ""
                for i in range(n - 1, -1, -1):
                    m = re.search(r"(\w+)\(", src[i]) if src[i].startswith("__device__") else None
                    if m:
                        fn = m.group(1)
                        break
                kind = {"sqrt_nr": "sqrt_nr", "sqrt_nr_ok": "sqrt_nr", "rcp_nr": "rcp_nr", "sqrt_rn": "exact sqrt fallback",
                        "sqrt_exact": "sqrt_nr", "inv_len": "vnorm/inv_len", "wave_any": "wave_any"}.get(fn, fn or "rt_common")
                break
            if f == SRC:
                hit = next((o for o, a, b in ops if a <= n <= b), None)
                if hit:
                    kind = hit
                    break
        tab[(phase, kind)] += 1
        tot[phase] += 1
    kinds = sorted({k for _, k in tab}, key=lambda k: -sum(v for (p, kk), v in tab.items() if kk == k))
    ph = ["query", "pass A", "pass B", "hit", "done", "loop control", "pass A (>1 light)", "prologue/epilogue"]
    print("%-20s" % "op \\ phase" + "".join("%10s" % p[:10] for p in ph) + "%10s" % "total")
    for k in kinds:
        row = [tab[(p, k)] for p in ph]
        print("%-20s" % k + "".join("%10d" % v for v in row) + "%10d" % sum(row))
    print("%-20s" % "total" + "".join("%10d" % tot[p] for p in ph) + "%10d" % sum(tot.values()))


if __name__ == "__main__":
    main()
