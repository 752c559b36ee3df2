"""One parameterised GPU session (run on the GPU box from the repo root through gpurun).

    python3 -u tools/gpu_session.py TAG STEP [STEP ...]

Each STEP runs as a child process under its own time limit, its output in gpurun_out/TAG_<n>.log;
the JSON lines it prints are echoed.  The session stops at the first step that fails (non-zero exit,
time limit, abort): nothing more runs on the GPU after a fault.  This process never touches the GPU
itself (no torch import), so it may start rocprofv3 as a child.

STEP forms (values after '=' separated by ':'):
  clock                         GPU clocks / power snapshot (amd-smi, else rocm-smi)
  pytest=EXPR                   python -m pytest tests -m gpu -k EXPR (EXPR 'all' = no -k)
  bench=CFG[:K[:W[:OPTS]]]      bench.py --config CFG --steps K --warmup W, no CPU baseline / extras;
                                OPTS = key=v+key=v (rt_set_option)
  benchfull                     the default bench.py run (what the driver records)
  smoke                         __graft_entry__.smoke()
  ab=CFGS:SPECS                 tools/ab_walk.py SPECS with AB_CFGS=CFGS (SPECS = name[@k=v+k=v]:block,...)
  abt=TILE:REPS:CFGS:SPECS      the same on rank 0's tile of a TILE-GPU run (rows 0::TILE), REPS frames timed
  tiles=CFG:NS[:SETS]           tools/occupancy_probe.py CFG NS "SETS" (SETS: k=v,k=v;k=v)
  kt=CFG[:OPTS[:STEPS]]         rocprofv3 --kernel-trace --stats of bench.py (STEPS steps, default 1, after 1
                                warmup) -> gpurun_out/TAG_kt_CFG
  pmc=CFG:GROUP[:OPTS[:STEPS]]  one rocprofv3 --pmc pass (GROUP: fetch, write, req, sq, hit, ta, stall) of bench.py
  py=SCRIPT[:ARGS]              python3 -u SCRIPT ARGS (ARGS split on '+')
  ktpy=NAME:SCRIPT[:ARGS]       rocprofv3 --kernel-trace --stats of a py step -> gpurun_out/TAG_kt_NAME
  pmcpy=NAME:GROUP:SCRIPT[:ARGS] one rocprofv3 --pmc pass of a py step -> gpurun_out/TAG_pmc_NAME_GROUP
  lib=NAME                      later steps load lib/variants/libNAME.so (ENSEM3A_RT_LIB; kt / pmc output names
                                get _NAME); lib=default goes back to the product library
Limits: LIMIT_<KIND> env overrides the default seconds of a step kind.
"""
import os
import shlex
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "gpurun_out")
PY = sys.executable or "python3"
LIMITS = {"clock": 30, "pytest": 900, "bench": 300, "benchfull": 600, "smoke": 180, "ab": 600, "abt": 600, "tiles": 400, "kt": 300,
          "pmc": 240, "py": 600, "ktpy": 400, "pmcpy": 240}
PMC = {
    "fetch": "FETCH_SIZE",
    "write": "WRITE_SIZE",
    "hit": "TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum TCC_EA0_WRREQ_64B_sum",
    "req": "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum",
    "stall": "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_INSTS_LDS "
             "SQ_INSTS_VALU GRBM_GUI_ACTIVE",
    "ta": "TA_TA_BUSY_sum SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_WAVE_CYCLES GRBM_GUI_ACTIVE",
    "sq": "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU "
          "SQ_WAIT_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE GRBM_COUNT",
}


def bench_args(cfg, steps="1", warmup="1", opts=""):
    a = [PY, "-u", "bench.py", "--config", cfg, "--steps", steps, "--warmup", warmup, "--no-cpu-baseline",
         "--no-extra"]
    for kv in filter(None, opts.split("+")):
        a += ["--option", kv]
    return a


def command(kind, val, tag, n):
    env = {}
    p = val.split(":") if val else []
    if kind == "clock":
        smi = ("amd-smi metric -c -p 2>/dev/null || rocm-smi --showclocks --showpower --showtemp 2>/dev/null "
               "|| echo no smi")
        return ["bash", "-c", smi], env
    if kind == "pytest":
        a = [PY, "-u", "-m", "pytest", "tests", "-m", "gpu", "-x", "-v", "-rP", "--timeout", "300", "--timeout-method",
             "thread"]
        if val and val != "all":
            a += ["-k", val]
        return a, env
    if kind == "bench":
        return bench_args(p[0], p[1] if len(p) > 1 else "2", p[2] if len(p) > 2 else "1",
                          p[3] if len(p) > 3 else ""), env
    if kind == "benchfull":
        return [PY, "-u", "bench.py"], env
    if kind == "smoke":
        return [PY, "-u", "-c", "import __graft_entry__ as g; g.smoke()"], env
    if kind == "ab":
        env["AB_CFGS"] = p[0]
        return [PY, "-u", "tools/ab_walk.py", ":".join(p[1:])], env
    if kind == "abt":   # abt=TILE:REPS:CFGS:SPECS -- ab on rank 0's tile of a TILE-GPU run, REPS frames timed
        env["AB_TILE"], env["AB_REPS"], env["AB_CFGS"] = p[0], p[1], p[2]
        return [PY, "-u", "tools/ab_walk.py", ":".join(p[3:])], env
    if kind == "tiles":
        return [PY, "-u", "tools/occupancy_probe.py", p[0], p[1], p[2] if len(p) > 2 else ""], env
    if kind in ("kt", "pmc"):
        cfg = p[0]
        opts = (p[2] if len(p) > 2 else "") if kind == "pmc" else (p[1] if len(p) > 1 else "")
        nst = (p[3] if len(p) > 3 else "1") if kind == "pmc" else (p[2] if len(p) > 2 else "1")
        lib = os.environ.get("ENSEM3A_RT_LIB")
        name = f"{tag}_{kind}_{cfg}" + (f"_{p[1]}" if kind == "pmc" else "") + \
            ("_" + "".join(ch if ch.isalnum() else "-" for ch in opts) if opts else "") + \
            ("_" + os.path.basename(lib)[3:-3] if lib else "")
        prof = ["rocprofv3"] + (["--kernel-trace", "--stats"] if kind == "kt" else ["--pmc"] + PMC[p[1]].split())
        return prof + ["--output-format", "csv", "-d", os.path.join(OUT, name), "-o", name, "--"] + \
            bench_args(cfg, nst or "1", "1", opts) + ["--no-counts"], env
    if kind == "py":
        return [PY, "-u", p[0]] + (p[1].split("+") if len(p) > 1 and p[1] else []), env
    if kind == "pmcpy":   # pmcpy=NAME:GROUP:SCRIPT[:ARGS] -- one --pmc pass (GROUP as pmc=) of a py step
        name = f"{tag}_pmc_{p[0]}_{p[1]}"
        return ["rocprofv3", "--pmc"] + PMC[p[1]].split() + ["--output-format", "csv", "-d", os.path.join(OUT, name),
                "-o", name, "--", PY, "-u", p[2]] + (p[3].split("+") if len(p) > 3 and p[3] else []), env
    if kind == "ktpy":
        name = f"{tag}_kt_{p[0]}"
        return ["rocprofv3", "--kernel-trace", "--stats", "--output-format", "csv", "-d", os.path.join(OUT, name),
                "-o", name, "--", PY, "-u", p[1]] + (p[2].split("+") if len(p) > 2 and p[2] else []), env
    raise SystemExit(f"unknown step kind {kind!r}")


def main():
    tag, steps = sys.argv[1], sys.argv[2:]
    os.makedirs(OUT, exist_ok=True)
    os.environ.setdefault("TMPDIR", "/tmp")
    for n, st in enumerate(steps):
        kind, _, val = st.partition("=")
        if kind == "lib":   # lib=NAME: later steps load lib/variants/libNAME.so (lib=default: the product library)
            if val == "default":
                os.environ.pop("ENSEM3A_RT_LIB", None)
            else:
                os.environ["ENSEM3A_RT_LIB"] = os.path.join(ROOT, "ensem3a_openclraytracer_amd", "lib", "variants",
                                                            f"lib{val}.so")
            print(f"== step {n}: {st}", flush=True)
            continue
        cmd, env = command(kind, val, tag, n)
        limit = int(os.environ.get("LIMIT_" + kind.upper(), LIMITS[kind]))
        log = os.path.join(OUT, f"{tag}_{n}_{kind}.log")
        print(f"== step {n}: {st} (limit {limit} s) -> {os.path.relpath(log, ROOT)}", flush=True)
        full = ["timeout", "-k", "10", str(limit)] + cmd
        with open(log, "w") as f:
            f.write(" ".join(shlex.quote(c) for c in full) + "\n")
            f.flush()
            r = subprocess.run(full, cwd=ROOT, env=dict(os.environ, **env), stdout=f, stderr=subprocess.STDOUT)
        with open(log, errors="replace") as f:
            lines = f.read().splitlines()
        shown = [ln for ln in lines if ln.startswith("{") or ln.startswith("FAILED") or " passed" in ln
                 or " failed" in ln or ln.startswith("GPU") or "MHz" in ln or "Mhz" in ln]
        for ln in shown[-40:]:
            print(ln[:900], flush=True)
        if r.returncode != 0:
            print(f"== step {n} FAILED rc={r.returncode}; last lines:", flush=True)
            for ln in lines[-25:]:
                print("   " + ln[:400], flush=True)
            sys.exit(1)
    print(f"== session {tag} done", flush=True)


if __name__ == "__main__":
    main()
