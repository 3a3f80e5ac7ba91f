"""No function reads a name that nothing defines (scripts/check_names.py).

A missing import in a path the CPU suite never runs -- `cli serve`'s engine
builder once read ``torch`` without importing it -- only failed on the GPU
box.  The checker catches that class of bug statically over every Python
file that ships or runs on the box."""
import importlib.util
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent


def _checker():
    spec = importlib.util.spec_from_file_location("check_names", ROOT / "scripts" / "check_names.py")
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_no_undefined_names():
    mod = _checker()
    files = []
    for d in ("llm_message_queue_amd", "bench", "scripts", "tests"):
        files += sorted((ROOT / d).rglob("*.py"))
    files += [ROOT / "bench.py", ROOT / "__graft_entry__.py"]
    assert mod.check(files) == []


def test_checker_flags_a_missing_import(tmp_path):
    p = tmp_path / "m.py"
    p.write_text("import os\n\ndef build(n):\n    return torch.zeros(n), os.sep\n")
    assert mod_findings(p) == [f"{p}:4: undefined name 'torch'"]


def mod_findings(p):
    return _checker().check([p])
