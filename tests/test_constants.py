"""The field constants of csrc/fe25519.h and the Legendre-symbol facts the
Elligator2 map of csrc/verify.h relies on (tools/check_*.py), on CPU."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(script):
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", script)],
                       capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stdout + r.stderr


def test_fe_constants():
    _run("check_fe_constants.py")


def test_elligator_case_analysis():
    _run("check_elligator_exceptions.py")
