"""Every SMER_* environment switch the product reads (C-ABI sources, package
Python, bench.py) is listed in DESIGN.md §9, so the runtime-switch table
stays complete as switches are added."""
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "smer_music_generation_amd")


def _sources():
    for d, exts in ((os.path.join(PKG, "csrc"), (".hip", ".cpp", ".h")), (PKG, (".py",))):
        for name in sorted(os.listdir(d)):
            if name.endswith(exts):
                yield os.path.join(d, name)
    yield os.path.join(ROOT, "bench.py")


def _switches():
    pat = re.compile(r'(?:getenv|environ\.get|environ\[)\(?\s*"(SMER_[A-Z0-9_]+)"')
    found = set()
    for path in _sources():
        with open(path) as f:
            found.update(pat.findall(f.read()))
    return found


def test_every_switch_is_documented():
    with open(os.path.join(ROOT, "DESIGN.md")) as f:
        design = f.read()
    table = design[design.index("## 9. Runtime switches"):]
    switches = _switches()
    assert len(switches) > 20
    missing = sorted(s for s in switches if "`%s`" % s not in table)
    assert not missing, "undocumented runtime switches: %s" % missing
