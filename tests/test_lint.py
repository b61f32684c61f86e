"""The tree passes its own blocking lint (CI's lint step, `tools/lint.py`)."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_lint_clean():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "lint.py")], capture_output=True, text=True,
                       cwd=ROOT)
    assert r.returncode == 0, r.stdout + r.stderr


def test_lint_catches_findings(tmp_path):
    bad = tmp_path / "bad.py"
    bad.write_text("import os\nimport sys\n\n\ndef f():\n    return sys.argv == None\n\n\ndef f():\n    pass\n")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "lint.py"), str(bad)], capture_output=True,
                       text=True)
    assert r.returncode == 1
    assert "'os' imported but unused" in r.stdout
    assert "redefinition of 'f'" in r.stdout
    assert "comparison to None" in r.stdout
