"""The library's environment knobs (csrc/host/tuning.cpp): read in one place,
each listed in INTEGRATION.md with a test, removed knobs named (CPU only)."""
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "cfd-demo2_amd", "csrc")


def _sources():
    for d, _, fs in os.walk(CSRC):
        for f in fs:
            if f.endswith((".cpp", ".hpp", ".hip", ".h")):
                p = os.path.join(d, f)
                yield p, open(p).read()


def _table():
    src = open(os.path.join(CSRC, "host", "tuning.cpp")).read()
    body = src[src.index("kKnobs[] = {"):src.index("static_assert")]
    return re.findall(r'"(CFD_[A-Z0-9_]+)"', body), src


def test_one_getenv_site():
    calls = {p: len(re.findall(r"\bgetenv\s*\(", s)) for p, s in _sources()}
    calls = {os.path.relpath(p, CSRC): n for p, n in calls.items() if n}
    assert calls == {os.path.join("host", "tuning.cpp"): 2}, calls  # knob() + the removed-knob scan


def test_knob_table_matches_integration_md():
    names, _ = _table()
    assert len(names) == len(set(names)) <= 12
    doc = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    sec = doc[doc.index("## Environment knobs"):]
    sec = sec[:sec.index("Removed in round 6")]
    documented = re.findall(r"^\| `(CFD_[A-Z0-9_]+)` \|", sec, re.M)
    assert documented == names
    # every knob is named by some GPU test
    tests = "".join(open(os.path.join(ROOT, "tests", f)).read()
                    for f in os.listdir(os.path.join(ROOT, "tests")) if f.startswith("test_gpu") or f in
                    ("test_voronoi.py", "test_watchdog.py"))
    for n in names:
        assert n in tests, f"{n} is not exercised by a GPU test"


def test_removed_knobs_are_not_read_and_are_named():
    names, src = _table()
    removed = re.findall(r'"(CFD_[A-Z0-9_]+)"', src[src.index("kRemoved[] = {"):src.index("void warn_removed_once")])
    assert not set(removed) & set(names)
    code = "".join(s for p, s in _sources() if not p.endswith("tuning.cpp"))
    for n in removed:
        assert f'"{n}"' not in code, f"{n} still read"
