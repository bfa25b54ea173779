"""bench.py's workload functions only run on a GPU box; this CPU check catches a name used in
one of them that nothing in scope defines (the slip that broke the FedDyn / SCAFFOLD lines once:
a JSON field copied in from another workload).  A small scope walk -- no pyflakes here."""
import ast
import builtins
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bound_names(node):
    """Every name a function binds anywhere inside it (parameters, assignments, loop and
    comprehension targets, imports, with / except targets, nested defs and their params)."""
    out = set()
    for n in ast.walk(node):
        if isinstance(n, (ast.FunctionDef, ast.AsyncFunctionDef, ast.Lambda)):
            a = n.args
            out.update(x.arg for x in a.args + a.kwonlyargs + a.posonlyargs)
            if a.vararg:
                out.add(a.vararg.arg)
            if a.kwarg:
                out.add(a.kwarg.arg)
            if not isinstance(n, ast.Lambda):
                out.add(n.name)
        elif isinstance(n, ast.Name) and isinstance(n.ctx, (ast.Store, ast.Del)):
            out.add(n.id)
        elif isinstance(n, (ast.Import, ast.ImportFrom)):
            out.update((a.asname or a.name).split(".")[0] for a in n.names)
        elif isinstance(n, ast.ExceptHandler) and n.name:
            out.add(n.name)
        elif isinstance(n, ast.ClassDef):
            out.add(n.name)
    return out


def _undefined(path):
    tree = ast.parse(open(path).read(), path)
    module = _bound_names(ast.Module(body=[n for n in tree.body if not isinstance(n, ast.FunctionDef)],
                                     type_ignores=[]))
    module.update(n.name for n in tree.body if isinstance(n, (ast.FunctionDef, ast.ClassDef)))
    module.update(("__file__", "__name__", "__doc__"))    # module attributes every module has
    bad = []
    for fn in (n for n in tree.body if isinstance(n, ast.FunctionDef)):
        local = _bound_names(fn)
        for n in ast.walk(fn):
            if isinstance(n, ast.Name) and isinstance(n.ctx, ast.Load):
                if n.id not in local and n.id not in module and not hasattr(builtins, n.id):
                    bad.append(f"{os.path.basename(path)}:{n.lineno} {fn.name}: {n.id}")
    return bad


def test_bench_functions_use_only_defined_names():
    assert _undefined(os.path.join(ROOT, "bench.py")) == []


def test_checker_catches_an_undefined_name(tmp_path):
    p = tmp_path / "m.py"
    p.write_text("X = 1\n\ndef f(a):\n    b = a + X\n    return {'t': traffic, 'b': b}\n")
    assert _undefined(str(p)) == ["m.py:5 f: traffic"]
