"""Every LDNN_* environment knob the package reads is listed in the README's knob table, and the
table lists nothing the code no longer reads (the table is the knob inventory)."""
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "learning-deep-neural-network-in-distributed-computing-environment_amd")
READ = re.compile(r'(?:environ\.get|getenv|env_int|environ\[)\(?"(LDNN_[A-Z0-9_]+)"')


def _read_knobs():
    files = [os.path.join(ROOT, "bench.py"), os.path.join(ROOT, "__graft_entry__.py")]
    for d, _, names in os.walk(PKG):
        files += [os.path.join(d, n) for n in names if n.endswith((".py", ".hip", ".cpp", ".h"))]
    found = set()
    for f in files:
        with open(f, encoding="utf-8", errors="replace") as fh:
            found |= set(READ.findall(fh.read()))
    return found


def _table_knobs():
    with open(os.path.join(ROOT, "README.md"), encoding="utf-8") as fh:
        text = fh.read()
    sec = text[text.index("## Environment knobs"):]
    sec = sec[:sec.index("\n## ", 4)] if "\n## " in sec[4:] else sec
    rows = re.findall(r"^\| `(LDNN_[A-Z0-9_]+)` \|", sec, flags=re.M)
    count = int(re.search(r"## Environment knobs \((\d+)", sec).group(1))
    return rows, count


def test_readme_knob_table_matches_the_code():
    code = _read_knobs()
    rows, count = _table_knobs()
    assert len(rows) == len(set(rows)), "duplicate rows"
    assert set(rows) == code, (sorted(code - set(rows)), sorted(set(rows) - code))
    assert count == len(rows) <= 30
