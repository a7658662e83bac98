#!/usr/bin/env python3
"""Rewrite the `<!-- fig:KEY -->` figures of README.md, DESIGN.md and INTEGRATION.md from the round's profiles
(tests/test_headline_figures.py formats them and checks the result). Each figure after a marker is replaced by the
profiles' value in the same shape (digits, decimal point, exponent and unit as the formatted value has them).
usage: python tools/update_figures.py [--dry-run]"""
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import test_headline_figures as thf  # noqa: E402


def shape(value):
    """A regex for a figure of the same shape as `value` (runs of digits generalised)."""
    return "".join(r"\d+" if p.isdigit() else re.escape(p) for p in re.findall(r"\d+|\D", value))


def main():
    src = thf._sources()
    dry = "--dry-run" in sys.argv
    for doc in thf.DOCS:
        path = os.path.join(ROOT, doc)
        text = open(path).read()

        def repl(m):
            key = m.group(1)
            new = src[key]
            rest = m.group(3)
            mm = re.match(shape(new), rest)
            if not mm:
                print(f"{doc}: {key}: no figure of shape {new!r} after the marker: {rest[:30]!r}")
                return m.group(0)
            if mm.group(0) != new:
                print(f"{doc}: {key}: {mm.group(0)} -> {new}")
            return m.group(0)[: m.start(3) - m.start(0)] + new + rest[mm.end():]

        out = re.sub(r"(?s)<!-- fig:([a-z0-9_]+) -->(\**)([^|\n<]*)", repl, text)
        if not dry and out != text:
            open(path, "w").write(out)


if __name__ == "__main__":
    main()
