"""The C opcode loop of the restricted decoder (flame_amd/csrc/pickle_vm.c) against its
specification, the Python loop (PayloadDecoder.load_py): same objects for valid payloads, the
same exception type for every mutated / truncated one, and no read outside the buffer
(payloads placed against an unmapped guard page, in a child process so a fault is a failure,
not a crash of the suite).  The payloads are flame update messages as the channel carries
them (cloudpickle.dumps, channel.py:203-218 / :321-325), protocols 2-5."""
import collections
import enum
import os
import pickle
import subprocess
import sys

import cloudpickle
import numpy as np
import torch

from flame_amd import ingest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


class Kind(enum.Enum):
    WEIGHTS = 1
    ROUND = 2


def _messages(seed, n):
    rng = np.random.default_rng(seed)
    dts = [torch.float32, torch.bfloat16, torch.float16, torch.float64, torch.int64, torch.int32, torch.int16,
           torch.int8, torch.uint8, torch.bool]
    out = []
    for i in range(n):
        w = collections.OrderedDict()
        for k in range(int(rng.integers(1, 6))):
            shape = tuple(int(x) for x in rng.integers(0, 6, size=int(rng.integers(0, 4))))
            t = torch.from_numpy(np.asarray(rng.standard_normal(shape) * 7, dtype=np.float32)).to(dts[int(rng.integers(len(dts)))])
            if t.dim() >= 2 and rng.random() < 0.3:
                t = t.transpose(0, 1)
            w[f"layer{k}.w"] = t
        if rng.random() < 0.3:     # a big tensor: its BINBYTES sits outside pickle frames
            w["fc.w"] = torch.from_numpy(rng.standard_normal(70_000).astype(np.float32))
        meta = {"n": int(rng.integers(-2**40, 2**40)), "x": float(rng.standard_normal()), "s": "tré-%d" % i,
                "l": [1, 2, (3, None, True)], "set": {1, 2}, "fz": frozenset({"a"}), "c": complex(1, -2),
                "big": 10**30 * (1 if i % 2 else -1), "b": bytes(range(i % 7))}
        out.append(({Kind.WEIGHTS: w, Kind.ROUND: i, "meta": meta, "alias": w}, [2, 3, 4, 5][i % 4]))
    return out


def _payloads(seed=0, n=24):
    return [cloudpickle.dumps(m, protocol=p) for m, p in _messages(seed, n)]


def _decode(payload, vm):
    """(kind, value): the decoded object, or the exception type the decoder raised."""
    saved = ingest._VM
    ingest._VM = vm
    try:
        return "ok", ingest.decode(payload, extra_globals=ingest.allow_enum(Kind))
    except Exception as e:  # noqa: BLE001 -- the TYPE is what is compared
        return "err", type(e)
    finally:
        ingest._VM = saved


def _canon(x, _path=()):
    """A comparable form of a decoded message (containers recursively; a container met again
    on its own path -- a cycle a mutated memo can build -- by its depth)."""
    if isinstance(x, (dict, list, tuple, set, frozenset)):
        for d, y in enumerate(_path):
            if y is x:
                return ("cycle", d)
        _path = _path + (x,)
    if isinstance(x, torch.Tensor):
        b = x.contiguous().reshape(-1).view(torch.uint8).numpy().tobytes() if x.numel() else b""
        return ("T", x.dtype, tuple(x.shape), x.stride(), x.storage_offset(), b)
    if isinstance(x, dict):
        return ("D", type(x).__name__, tuple((_canon(k, _path), _canon(v, _path)) for k, v in x.items()))
    if isinstance(x, (list, tuple)):
        return (type(x).__name__, tuple(_canon(v, _path) for v in x))
    if isinstance(x, (set, frozenset)):
        return (type(x).__name__, tuple(sorted(map(repr, x))))
    if isinstance(x, float) and x != x:
        return ("nan",)
    if isinstance(x, ingest._Span):
        return ("span", x.start, x.n)
    return (type(x).__name__, x)


def test_c_vm_is_the_default_and_built():
    assert ingest._VM is not None, "flame_amd._pickle_vm not built (python -m flame_amd.build)"


def test_c_vm_equals_python_vm_on_messages():
    vm = ingest._VM
    for pl in _payloads():
        a, b = _decode(pl, vm), _decode(pl, None)
        assert a[0] == b[0] == "ok", (a, b)
        assert _canon(a[1]) == _canon(b[1])
        ref = cloudpickle.loads(pl)
        assert _canon(a[1]["meta"]) == _canon(ref["meta"])
        assert a[1]["alias"] is a[1][Kind.WEIGHTS]          # memo: shared objects stay shared


def test_c_vm_equals_python_vm_on_mutations():
    """Byte flips, truncations, insertions, deletions: both loops agree on every outcome."""
    vm = ingest._VM
    rng = np.random.default_rng(5)
    pls = [p for p in _payloads(1, 12) if len(p) < 20_000]
    n_ok = n_err = 0
    for trial in range(1500):
        pl = bytearray(pls[trial % len(pls)])
        kind = trial % 4
        i = int(rng.integers(len(pl)))
        if kind == 0:
            pl[i] = int(rng.integers(256))
        elif kind == 1:
            del pl[i:]
        elif kind == 2:
            pl[i:i] = bytes(rng.integers(0, 256, size=int(rng.integers(1, 4)), dtype=np.uint8))
        else:
            del pl[i:i + int(rng.integers(1, 4))]
        pl = bytes(pl)
        a, b = _decode(pl, vm), _decode(pl, None)
        assert a[0] == b[0], (trial, a, b)
        if a[0] == "ok":
            n_ok += 1
            assert _canon(a[1]) == _canon(b[1]), trial
        else:
            n_err += 1
            assert a[1] is b[1], (trial, a[1], b[1])
    assert n_ok > 50 and n_err > 500          # both outcomes exercised


def test_storage_head_equals_the_python_record_parser():
    """storage_head (C) == _parse_storage_record (regex + field parser) on torch's own streams
    and on every single-byte corruption of one."""
    import io
    import warnings
    vm = ingest._VM
    for dt in (torch.float32, torch.bfloat16, torch.int64, torch.bool, torch.uint8):
        for n in (0, 1, 300, 70_000):
            bio = io.BytesIO()
            with warnings.catch_warnings():
                warnings.simplefilter("ignore")
                torch.save(torch.zeros(n, dtype=dt).storage(), bio, _use_new_zipfile_serialization=False)
            s = bio.getvalue()
            dec = ingest.PayloadDecoder(s)
            dec._storage_from_span(ingest._Span(0, len(s)))     # validates + caches the header
            hdr = next(h for h in ingest._STORAGE_HEADERS if s.startswith(h))
            got = vm.storage_head(memoryview(s), 0, len(s), ingest._STORAGE_HEADERS)
            exp = ingest._parse_storage_record(memoryview(s), len(hdr))
            assert got is not None and ingest._STORAGE_DTYPES[got[0]] == exp[0] and got[1:] == exp[1:]
            rec_end = exp[2]
            for i in range(len(hdr), rec_end):
                for v in (0, 0x71, 0xFF, s[i] ^ 1):
                    m = bytearray(s)
                    m[i] = v
                    m = bytes(m)
                    g = vm.storage_head(memoryview(m), 0, len(m), ingest._STORAGE_HEADERS)
                    e = ingest._parse_storage_record(memoryview(m), len(hdr))
                    if g is None or g[0] not in ingest._STORAGE_DTYPES:
                        continue        # C declined (or no such storage type): the Python path decides
                    assert e is not None and ingest._STORAGE_DTYPES.get(g[0]) == e[0] and g[1:] == e[1:], (dt, n, i, v)


def test_no_read_past_the_buffer_guard_page():
    """Every prefix of a payload, and mutations, decoded from a buffer that ends against a
    PROT_NONE page: the C loop must raise, never fault (child process)."""
    r = subprocess.run([sys.executable, os.path.join(HERE, "pickle_vm_guard.py")], cwd=ROOT,
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, (r.returncode, r.stdout[-2000:], r.stderr[-2000:])
    assert "guard ok" in r.stdout


def test_guard_page_run_under_ubsan(tmp_path):
    """The same run with the C loop built with -fsanitize=undefined (no recovery): any
    undefined behaviour (overflowing shifts, misaligned or null access) aborts the child."""
    import sysconfig
    from flame_amd import build as B
    lib = str(tmp_path / ("_pickle_vm" + sysconfig.get_config_var("EXT_SUFFIX")))
    subprocess.check_call(["gcc", "-O1", "-g", "-std=c11", "-shared", "-fPIC", "-fsanitize=undefined",
                           "-fno-sanitize-recover=all", f"-I{sysconfig.get_paths()['include']}", "-o", lib, B.VM_SRC])
    r = subprocess.run([sys.executable, os.path.join(HERE, "pickle_vm_guard.py"), "--lib", lib], cwd=ROOT,
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0 and "runtime error" not in r.stderr, (r.returncode, r.stdout[-2000:], r.stderr[-3000:])
    assert "guard ok" in r.stdout


def test_under_asan(tmp_path):
    """The guard-page fuzz and the differential tests with the C loop built with
    -fsanitize=address,undefined, inside an ASan-linked embedded CPython (tests/asan/py_embed.c)
    with PYTHONMALLOC=malloc, so the loop's own stack / mark arrays and every object it makes
    are ASan-checked heap."""
    import sysconfig
    from flame_amd import build as B
    inc = sysconfig.get_paths()["include"]
    libdir = sysconfig.get_config_var("LIBDIR")
    ver = sysconfig.get_config_var("LDVERSION")
    san = ["-g", "-O1", "-fsanitize=address,undefined", "-fno-omit-frame-pointer", "-fno-sanitize-recover=all"]
    exe = str(tmp_path / "py_embed")
    lib = str(tmp_path / ("_pickle_vm" + sysconfig.get_config_var("EXT_SUFFIX")))
    subprocess.check_call(["gcc", *san, os.path.join(HERE, "asan", "py_embed.c"), f"-I{inc}", f"-L{libdir}",
                           f"-lpython{ver}", "-lcrypt", "-ldl", "-lm", "-o", exe])
    subprocess.check_call(["gcc", *san, "-std=c11", "-shared", "-fPIC", f"-I{inc}", "-o", lib, B.VM_SRC])
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:detect_odr_violation=0:abort_on_error=1",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1", PYTHONMALLOC="malloc")
    r = subprocess.run([exe, os.path.join(HERE, "asan", "run_pickle_vm.py"), lib], cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=900)
    assert r.returncode == 0 and "ERROR: AddressSanitizer" not in r.stderr and "runtime error" not in r.stderr, \
        (r.returncode, r.stdout[-2000:], r.stderr[-4000:])
    assert "asan run ok" in r.stdout


def test_refusals_are_identical():
    """Globals outside the allowlist, BUILD with state, persistent ids: refused by both loops
    with the same error (nothing executed)."""
    class Evil:
        def __reduce__(self):
            return (os.system, ("true",))
    bad = [pickle.dumps(Evil(), protocol=p) for p in (2, 4, 5)]
    bad.append(pickle.dumps(collections.Counter(a=1), protocol=4))        # BUILD / non-allowlisted
    bad.append(b"\x80\x04\x95\x05\x00\x00\x00\x00\x00\x00\x00N\x51.")         # BINPERSID
    # bytes / bytearray rebuilt from a size (n zero bytes allocated on the sender's say-so)
    bad.append(b"\x80\x02c__builtin__\nbytearray\nJ\x00\x00\x00\x40\x85R.")
    bad.append(b"\x80\x03cbuiltins\nbytes\nJ\x00\x00\x00\x40\x85R.")
    for pl in bad:
        a, b = _decode(pl, ingest._VM), _decode(pl, None)
        assert a == b == ("err", pickle.UnpicklingError), (pl, a, b)
    # ... while the forms pickles actually use still decode
    for v in (b"", bytearray(b"xyz"), b"\x00\xff" * 5):
        for proto in (2, 3, 5):
            pl = pickle.dumps({"v": v}, protocol=proto)
            for vm in (ingest._VM, None):
                got = _decode(pl, vm)
                assert got[0] == "ok" and got[1]["v"] == v and type(got[1]["v"]) is type(v), (v, proto, got)
