"""DESIGN.md cites its numbers' sources as `profiles/...` paths: every path it
names must exist in the tree (globs allowed), so a moved or deleted profile shows up here."""
import glob
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_design_cites_existing_profiles():
    text = open(os.path.join(ROOT, 'DESIGN.md')).read()
    paths = sorted(set(re.findall(r'profiles/[A-Za-z0-9_./*{},-]+', text)))
    assert paths
    missing = []
    for p in paths:
        p = p.rstrip('.,')
        if '{' in p:  # brace lists: check each alternative
            head, alts, tail = re.match(r'(.*)\{([^}]*)\}(.*)', p).groups()
            cands = [head + a + tail for a in alts.split(',')]
        else:
            cands = [p]
        for c in cands:
            if not glob.glob(os.path.join(ROOT, c)):
                missing.append(c)
    assert not missing, missing


def test_design_is_a_current_state_document():
    lines = open(os.path.join(ROOT, 'DESIGN.md')).read().splitlines()
    assert len(lines) <= 520, len(lines)
