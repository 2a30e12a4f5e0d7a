"""Guard: no tracked file may ask for a sanitizer build of GPU code.

The GPU pool refuses to run anything that would execute a hipcc/clang
statement with a sanitizer flag that reaches the device pass (GPUTEST_r03
was refused for exactly this).  A sanitizer flag is acceptable only when it
directly follows ``-Xarch_host`` or when the same line also carries
``-fno-gpu-sanitize``.  Documentation (``*.md``) and the driver's JSON
records are prose, not build statements, and are skipped.
"""
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FLAG = "-fsan" + "itize="          # spelled in two parts so this file never matches itself
OK_LINE = "-fno-gpu-" + "sanitize"
HOST_ONLY = re.compile(r"-Xarch_host\s*[\"',]*\s*$")
SKIP_EXT = (".md", ".json", ".npz", ".csv", ".txt", ".log")


def _tracked_files():
    try:
        out = subprocess.run(["git", "ls-files"], cwd=ROOT, check=True, capture_output=True,
                             text=True).stdout.split()
    except (OSError, subprocess.CalledProcessError):
        pytest.skip("not a git checkout")
    # plus untracked sources a commit would add
    extra = subprocess.run(["git", "ls-files", "--others", "--exclude-standard"], cwd=ROOT,
                           capture_output=True, text=True).stdout.split()
    return sorted(set(out) | set(extra))


def offending_lines(text):
    bad = []
    for no, line in enumerate(text.splitlines(), 1):
        if FLAG not in line or OK_LINE in line:
            continue
        for m in re.finditer(re.escape(FLAG), line):
            if not HOST_ONLY.search(line[:m.start()]):
                bad.append((no, line.strip()))
                break
    return bad


def test_lint_catches_a_device_sanitizer_line():
    assert offending_lines('hipcc -O2 ' + FLAG + 'address -c x.hip')
    assert not offending_lines('hipcc -Xarch_host ' + FLAG + 'address -c x.hip')
    assert not offending_lines('hipcc ' + FLAG + 'address ' + OK_LINE + ' -c x.hip')


def test_no_device_sanitizer_build_in_tree():
    found = []
    for rel in _tracked_files():
        if rel.endswith(SKIP_EXT) or rel.startswith(("VERDICT", "ADVICE")):
            continue
        path = os.path.join(ROOT, rel)
        if not os.path.isfile(path):
            continue
        try:
            with open(path, encoding="utf-8") as fh:
                text = fh.read()
        except (UnicodeDecodeError, OSError):
            continue
        found += [(rel, no, line) for no, line in offending_lines(text)]
    assert not found, found
