"""The product path has no CPU fallback: without libksched.so it fails loudly,
and nothing in the shipped package or library sources reaches the oracle."""
import os
import re
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
PKG = ROOT / "k8s-1m_amd"


def test_missing_library_raises_import_error(tmp_path):
    code = ("import sys; sys.path.insert(0, %r)\n"
            "from ksched import Scheduler\n"
            "try:\n"
            "    Scheduler(16)\n"
            "except ImportError as e:\n"
            "    print('IMPORT-ERROR', e)\n"
            "    sys.exit(0)\n"
            "sys.exit(3)\n") % str(PKG)
    env = dict(os.environ, KSCHED_LIB_DIR=str(tmp_path / "absent"))
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "IMPORT-ERROR" in r.stdout and "libksched.so is missing" in r.stdout


def test_product_sources_never_reference_the_oracle():
    pat = re.compile(r"\boracle\b|pyoracle|liboracle", re.IGNORECASE)
    hits = []
    for p in list(PKG.rglob("*.py")) + list(PKG.rglob("*.cpp")) + list(PKG.rglob("*.hip")) + \
            list(PKG.rglob("*.hpp")) + list((ROOT / "include").glob("*.h")) + [PKG / "Makefile"]:
        if not p.exists() or "__pycache__" in p.parts:
            continue
        for i, line in enumerate(p.read_text(errors="replace").splitlines(), 1):
            code = line.split("//")[0].split("#")[0] if p.suffix != ".py" else line.split("#")[0]
            if pat.search(code) and not code.lstrip().startswith(("*", '"""', "'")):
                hits.append(f"{p.relative_to(ROOT)}:{i}: {line.strip()}")
    assert not hits, "product code references the oracle:\n" + "\n".join(hits)
