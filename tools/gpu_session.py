#!/usr/bin/env python3
"""One GPU session on the MI355X box: named steps run one after another, each under its own time
limit, output in gpurun_out/<tag>_<step>.log; the session stops at the first step that fails,
times out or crashes (no retries, nothing else touches the GPU after a fault).  Replaces round 5's
thirty one-off tools/gpu_r05_*.sh scripts.

    gpurun --timeout 1100 -- python3 tools/gpu_session.py r06a probe chain_bf16 e2e_shm
    python3 tools/gpu_session.py --list

The parent never initialises the GPU (every step is a child process, never an exec).  A step is
a command line (run from the repository root) and a time limit; ``{key}`` fields are filled from
``--set key=value`` (defaults in PARAMS).  Summaries worth keeping are copied into profiles/
afterwards (tools/README.md).
"""
import argparse
import os
import shlex
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PY = sys.executable or "python3"
AB = "build/ab/variants/lib_r05_step.so"     # the round-5 step (tools/kernel_sweep.py --build --variants r05_step)
PARAMS = {"clients": "64", "params": "2000000", "steps": "10", "warmup": "3", "offsets": "0,4,356",
          "seed_offset": "300000"}

# name -> (seconds, command).  Commands are lists; "rocprof:" prefixes run under rocprofv3 stats.
STEPS = {
    "pytest_gpu": (1000, [PY, "-u", "-m", "pytest", "tests", "-m", "gpu", "-x", "-q", "--timeout", "300",
                          "--timeout-method", "thread", "--durations", "5"]),
    "pytest_slab": (300, [PY, "-u", "-m", "pytest", "tests/test_gpu_slab_write.py", "tests/test_gpu_shm.py", "-m", "gpu",
                          "-x", "-q", "--timeout", "200", "--timeout-method", "thread"]),
    "pytest_shard": (400, [PY, "-u", "-m", "pytest", "tests/test_gpu_shard.py", "-m", "gpu", "-x", "-q", "--timeout",
                           "200", "--timeout-method", "thread"]),
    "pytest_chain": (400, [PY, "-u", "-m", "pytest", "tests/test_gpu_eager_fedopt_chain.py",
                           "tests/test_gpu_fastmath.py", "tests/test_gpu_dtype_matrix.py", "-m", "gpu", "-x", "-q",
                           "--timeout", "200", "--timeout-method", "thread"]),
    "smoke": (300, [PY, "-c", "import __graft_entry__ as g; g.smoke(); print('smoke ok')"]),
    "bench_default": (300, [PY, "bench.py"]),
    "probe": (300, [PY, "tools/fp_probe.py"]),
    "h2d_paths": (200, [PY, "tools/h2d_paths.py", "--offsets", "{offsets}"]),
    "ingest_diag": (300, [PY, "tools/ingest_diag.py"]),
    # eager FedOPT chain, 64 x 25M: the shipped library against the round-5 step, one process, bitwise
    **{f"chain_{v}_{dt}": (400, [PY, "tools/chain_sweep.py", "--variant", f"fed{v}", "--dtype", dt, "--rounds", "6",
                                  "--libs", f"flame_amd/libflame_amd.so,{AB}"])
       for v in ("adam", "yogi", "adagrad") for dt in ("f32", "bf16", "f16")},
    **{f"eager_{v}": (300, [PY, "bench.py", "--workload", f"fed{v}_eager"]) for v in ("adam", "yogi", "adagrad")},
    # the 16-bit steps' admission (FLAME_T_HALF_ADMIT) against the fp32 step's, one process, bitwise, over
    # enough rounds for stalled weights' m to decay through [2^-133, 2^-85] (bf16)
    **{f"chain_admit_{v}_{dt}": (400, [PY, "tools/chain_sweep.py", "--variant", f"fed{v}", "--dtype", dt, "--rounds",
                                       "18", "--libs", "flame_amd/libflame_amd.so,build/ab/variants/lib_r06_admit.so"])
       for v in ("adam", "yogi", "adagrad") for dt in ("bf16", "f16")},
    # the fp16 chain on packed halves against the fp32-register step, one process, bitwise
    **{f"chain_native_{v}": (400, [PY, "tools/chain_sweep.py", "--variant", f"fed{v}", "--dtype", "f16", "--rounds",
                                   "8", "--libs", "flame_amd/libflame_amd.so,build/ab/variants/lib_r06_f16.so"])
       for v in ("adam", "yogi", "adagrad")},
    # the packed-fp16 body's v_sqrt_f16 root and fp16 numerators against its first version (commit
    # 828bb82's source, built into build/ab/variants/lib_r06_f16a.so), one process, bitwise
    **{f"chain_f16a_{v}": (400, [PY, "tools/chain_sweep.py", "--variant", f"fed{v}", "--dtype", "f16", "--rounds",
                                 "8", "--libs", "flame_amd/libflame_amd.so,build/ab/variants/lib_r06_f16a.so"])
       for v in ("adam", "yogi", "adagrad")},
    # fresh random 16-bit eager cases (the packed-fp16 chain body against the per-call launches)
    "soak_eager16": (600, ["env", "FLAME_RANDOM_SCALE=50", "FLAME_RANDOM_SEED_OFFSET=200000", PY, "-u", "-m",
                           "pytest", "tests/test_gpu_random_cases.py", "-m", "gpu", "-k", "eager_fedopt_16bit", "-x",
                           "-q", "--timeout", "200", "--timeout-method", "thread"]),
    # the keys the fused kernels do not take, as flame_elementwise programs, and every suite that
    # reaches them (mixed / narrow / int / fp64 keys of FedAvg, FedOPT, FedBuff, FedDyn, SCAFFOLD)
    "pytest_ew": (600, [PY, "-u", "-m", "pytest", "tests/test_gpu_elementwise.py", "tests/test_gpu_dtype_matrix.py",
                        "tests/test_gpu_parity.py", "tests/test_gpu_random_cases.py", "-m", "gpu", "-x", "-q",
                        "--timeout", "200", "--timeout-method", "thread"]),
    # fresh random cases through every optimizer (mixed / int / fp64 keys reach flame_elementwise)
    "soak_random": (900, ["env", "FLAME_RANDOM_SCALE=6", "FLAME_RANDOM_SEED_OFFSET={seed_offset}", PY, "-u", "-m", "pytest",
                          "tests/test_gpu_random_cases.py", "-m", "gpu", "-k",
                          "random_case_vs_oracle or random_stateful or random_hierarchy", "-x", "-q", "--timeout",
                          "300", "--timeout-method", "thread"]),
    "ew_overhead": (200, [PY, "tools/ew_overhead.py"]),
    "ew_fp64": (200, [PY, "tools/ew_overhead.py", "--fp64"]),
    "pytest_f16": (400, [PY, "-u", "-m", "pytest", "tests/test_gpu_f16_chain_edges.py", "tests/test_gpu_half_admission.py",
                         "tests/test_gpu_eager_fedopt_chain.py", "-m", "gpu", "-x", "-v", "--timeout", "200",
                         "--timeout-method", "thread"]),
    "pytest_half": (400, [PY, "-u", "-m", "pytest", "tests/test_gpu_half_admission.py", "-m", "gpu", "-x", "-v",
                          "--timeout", "200", "--timeout-method", "thread"]),
    # the three variants interleaved in ONE process (Yogi within 3 % of Adam)
    **{f"chain_variants_{dt}": (400, [PY, "tools/chain_sweep.py", "--variant", "fedadam,fedyogi,fedadagrad",
                                      "--dtype", dt, "--rounds", "6", "--libs", "flame_amd/libflame_amd.so"])
       for dt in ("f32", "bf16", "f16")},
    # end-to-end rows, 64 clients x 25M fp32 from host memory back to host memory
    **{f"e2e_{m}": (400, [PY, "bench.py", "--e2e", "--e2e-mode", m])
       for m in ("zerocopy", "copy", "pageable", "shm", "shm_reference", "eager", "shard", "shm_shard", "wire",
                 "wire_reference")},
    # the N-GPU end-to-end line rehearsed with gloo ranks sharing the box's one GPU
    **{f"e2e_shm_gloo{n}{suf}": (600, ["env", "FLAME_BENCH_BACKEND=gloo", PY, "bench.py", "--gpus", str(n), "--e2e",
                                       "--e2e-mode", "shm", "--e2e-egress", eg, "--clients", "{clients}", "--params",
                                       "{params}"])
       for n in (2, 8) for suf, eg in (("", "sharded"), ("_gathered", "gathered"))},
    **{f"e2e_shm_shard{suf}": (400, [PY, "bench.py", "--e2e", "--e2e-mode", "shm_shard", "--e2e-egress", eg])
       for suf, eg in (("_sharded_egress", "sharded"), ("_gathered", "gathered"))},
    **{f"sharded_gloo{n}": (600, ["env", "FLAME_BENCH_BACKEND=gloo", PY, "bench.py", "--gpus", str(n), "--clients",
                                  "{clients}", "--params", "{params}"]) for n in (2, 8)},
    **{f"hier_gloo{n}": (600, ["env", "FLAME_BENCH_BACKEND=gloo", PY, "bench.py", "--gpus", str(n), "--workload",
                               "hier_fedbuff", "--clients", "256", "--params", "{params}"]) for n in (2,)},
    "force_shard": (300, [PY, "bench.py", "--force-shard"]),
    # plain bench lines of the secondary paths (DESIGN §0's second table)
    **{f"line_{w}": (300, [PY, "bench.py", "--cpu-clients", "0", *a]) for w, a in {
        "c2": ["--clients", "256", "--params", "1000000", "--steps", "50", "--warmup", "5"],
        "fedavg_eager": ["--workload", "fedavg_eager", "--steps", "10", "--warmup", "3"],
        "scaffold": ["--workload", "scaffold", "--steps", "10", "--warmup", "3"],
        "hier_fetched": ["--workload", "hier_fedbuff", "--hier-middles", "fetched", "--steps", "10", "--warmup", "3"],
        "hier_sync": ["--workload", "hier_fedbuff", "--hier-mode", "sync", "--steps", "10", "--warmup", "3"]}.items()},
    # the evidence collection (round 5's gpu_r05_prof.sh): each default path's bench line under
    # rocprofv3 --kernel-trace --stats (the SAME process's kernel summary) ...
    **{f"prof_{w}": (400, ["rocprof:", PY, "bench.py", *a]) for w, a in {
        "fedavg": ["--steps", "20", "--warmup", "5"],
        "fedadam": ["--workload", "fedadam", "--steps", "10", "--warmup", "3", "--cpu-clients", "16"],
        "fedyogi": ["--workload", "fedyogi", "--steps", "10", "--warmup", "3", "--cpu-clients", "0"],
        "fedadagrad": ["--workload", "fedadagrad", "--steps", "10", "--warmup", "3", "--cpu-clients", "0"],
        "hier_fedbuff": ["--workload", "hier_fedbuff", "--steps", "10", "--warmup", "3", "--cpu-clients", "0"],
        "fedbuff": ["--workload", "fedbuff", "--steps", "10", "--warmup", "3", "--cpu-clients", "0"],
        "fedadam_eager": ["--workload", "fedadam_eager", "--steps", "10", "--warmup", "3"],
        "fedyogi_eager": ["--workload", "fedyogi_eager", "--steps", "10", "--warmup", "3"],
        "fedadagrad_eager": ["--workload", "fedadagrad_eager", "--steps", "10", "--warmup", "3"],
        "feddyn": ["--workload", "feddyn", "--steps", "6", "--warmup", "2", "--cpu-clients", "0"]}.items()},
    # the eager lines at 16-bit dtypes (bench.py --dtype): line + CPU baseline under rocprofv3 stats
    **{f"prof_{v}_eager_{dt}": (400, ["rocprof:", PY, "bench.py", "--workload", f"fed{v}_eager", "--dtype", dt,
                                      "--steps", "10", "--warmup", "3"])
       for v in ("adam", "yogi", "adagrad") for dt in ("bf16", "f16")},
    **{f"pmc_{v}_eager_{dt}_{c}": (120, ["pmc:", c, "fedopt_chain", PY, "bench.py", "--workload", f"fed{v}_eager",
                                         "--dtype", dt, "--steps", "3", "--warmup", "1", "--cpu-clients", "0"])
       for v in ("adam", "yogi", "adagrad") for dt in ("bf16", "f16") for c in ("FETCH_SIZE", "WRITE_SIZE")},
    "prof_chain_bf16": (300, ["rocprof:", PY, "tools/chain_sweep.py", "--variant", "fedadam,fedyogi,fedadagrad",
                              "--dtype", "bf16", "--rounds", "3", "--libs", "flame_amd/libflame_amd.so"]),
    # ... and PMC passes, one counter per run (no trace domains), for the HBM traffic of a kernel
    **{f"pmc_{w}_{c}": (120, ["pmc:", c, rx, PY, "bench.py", *a, "--steps", "3", "--warmup", "1", "--cpu-clients", "0"])
       for w, rx, a in (("fedavg", "agg_reduce", []),
                        ("fedadam_eager", "fedopt_chain", ["--workload", "fedadam_eager"]),
                        ("fedyogi_eager", "fedopt_chain", ["--workload", "fedyogi_eager"]),
                        ("fedadagrad_eager", "fedopt_chain", ["--workload", "fedadagrad_eager"]),
                        ("hier_fedbuff", "hier_fedbuff", ["--workload", "hier_fedbuff"]))
       for c in ("FETCH_SIZE", "WRITE_SIZE")},
    **{f"pmc_chain_{dt}_{lb}_{c.split()[0]}": (120, ["pmc:", c, "fedopt_chain", PY, "tools/chain_sweep.py",
                                                     "--variant", "fedadam", "--dtype", dt, "--rounds", "1", "--libs",
                                                     lib])
       for dt in ("f32", "bf16", "f16") for lb, lib in (("r06", "flame_amd/libflame_amd.so"), ("r05", AB))
       for c in ("FETCH_SIZE", "WRITE_SIZE", "SQ_INSTS_VALU SQ_WAVES")},
}


def expand(cmd, params, tag, name):
    out = [c.format(**params) for c in cmd]
    d = os.path.join("gpurun_out", tag, name)
    if out and out[0] == "rocprof:":
        out = ["rocprofv3", "--kernel-trace", "--stats", "--output-format", "csv", "-d", d, "-o", "run", "--"] + out[1:]
    elif out and out[0] == "pmc:":
        counters, rx = out[1].split(), out[2]
        out = ["rocprofv3", "--pmc", *counters, "--kernel-include-regex", rx, "--output-format", "csv", "-d", d,
               "-o", "run", "--"] + out[3:]
    return out


def tidy(tag, name):
    """Drop a kernel-trace run's per-dispatch CSV (MBs); its stats summary stays."""
    d = os.path.join("gpurun_out", tag, name)
    for root, _, files in os.walk(d):
        for f in files:
            if f.endswith("kernel_trace.csv"):
                os.remove(os.path.join(root, f))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("tag", nargs="?")
    ap.add_argument("steps", nargs="*")
    ap.add_argument("--set", action="append", default=[], help="key=value for {key} fields")
    ap.add_argument("--list", action="store_true")
    a = ap.parse_args()
    if a.list or not a.tag:
        for nm, (lim, cmd) in STEPS.items():
            print(f"{nm:22s} {lim:5d} s  {' '.join(cmd)}")
        return 0
    params = dict(PARAMS)
    for kv in a.set:
        k, v = kv.split("=", 1)
        params[k] = v
    unknown = [s for s in a.steps if s not in STEPS]
    if unknown:
        print(f"gpu_session: unknown step(s) {unknown}; --list shows them", file=sys.stderr)
        return 2
    os.chdir(os.environ.get("GRAFT_REPO_ROOT", ROOT))
    os.makedirs("gpurun_out", exist_ok=True)
    env = dict(os.environ, PYTHONDONTWRITEBYTECODE="1", MASTER_ADDR="127.0.0.1", TMPDIR="/tmp")
    for name in a.steps:
        lim, cmd = STEPS[name]
        argv = expand(cmd, params, a.tag, name)
        log = os.path.join("gpurun_out", f"{a.tag}_{name}.log")
        t0 = time.time()
        with open(log, "w") as f:
            f.write("$ " + " ".join(shlex.quote(x) for x in argv) + "\n")
            f.flush()
            rc = subprocess.call(["timeout", "-k", "10", str(lim)] + argv, stdout=f, stderr=subprocess.STDOUT, env=env)
        tidy(a.tag, name)
        tail = open(log).read().splitlines()[-4:]
        print(f"[{a.tag}] {name}: rc={rc} {time.time() - t0:.0f} s", flush=True)
        for ln in tail:
            print("    " + ln[:400], flush=True)
        if rc != 0:       # a failure, a time limit (124 / 137), an abort or a fault: nothing more on the GPU
            print(f"[{a.tag}] stopping after {name} (rc={rc})", flush=True)
            return rc
    return 0


if __name__ == "__main__":
    sys.exit(main())
