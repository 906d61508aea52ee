"""bench.py's GPU-only paths (node files, API, flagship) cannot run on the CPU tier, so a name a function
uses but never defines or imports would only fail on the GPU box. Every free name of every function must
be a module-level name or a builtin."""
import builtins
import os
import symtable

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_names(path):
    src = open(path).read()
    top = symtable.symtable(src, path, "exec")
    module = {s.get_name() for s in top.get_symbols() if s.is_assigned() or s.is_imported()}
    known = module | set(dir(builtins)) | {"__file__", "__name__", "__doc__", "__spec__", "__loader__", "__package__"}
    bad = []

    def walk(t):
        for ch in t.get_children():
            for s in ch.get_symbols():
                if s.is_referenced() and s.is_global() and s.get_name() not in known:
                    bad.append(f"{ch.get_name()}: {s.get_name()}")
            walk(ch)

    walk(top)
    return bad


def test_bench_py_has_no_undefined_names():
    assert _free_names(os.path.join(ROOT, "bench.py")) == []


def test_tools_have_no_undefined_names():
    bad = []
    for name in ("tools/cold_task_bench.py", "tools/gpu_run.py", "benchmarks/run_configs.py"):
        bad += [f"{name}: {b}" for b in _free_names(os.path.join(ROOT, name))]
    assert bad == []
