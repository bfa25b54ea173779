"""Run inside tests/asan/py_embed (an ASan + UBSan embedded CPython, PYTHONMALLOC=malloc):
install the ASan build of the C decoder loop as flame_amd._pickle_vm, then run the guard-page
fuzz and the differential tests of tests/test_pickle_vm.py against it."""
import importlib.util
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [ROOT, os.path.dirname(HERE)]
spec = importlib.util.spec_from_file_location("flame_amd._pickle_vm", sys.argv[1])
mod = importlib.util.module_from_spec(spec)
spec.loader.exec_module(mod)
sys.modules["flame_amd._pickle_vm"] = mod
from flame_amd import ingest  # noqa: E402

ingest._VM = mod
import pickle_vm_guard  # noqa: E402
import test_pickle_vm as T  # noqa: E402

pickle_vm_guard.main()
T.test_c_vm_equals_python_vm_on_messages()
T.test_c_vm_equals_python_vm_on_mutations()
T.test_storage_head_equals_the_python_record_parser()
T.test_refusals_are_identical()
print("asan run ok", flush=True)
