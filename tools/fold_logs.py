"""Fold a round's short regression logs into one file (profiles/<round>/LOGS.md).

usage: python tools/fold_logs.py profiles/r03 [max_lines]

Every *.log directly in the directory with at most max_lines (default 30) lines becomes one
section of LOGS.md, headed by its old file name, under a summary table (file, lines, its last
non-empty line -- for a bench or test log, the result line).  The folded files are removed and
every reference to "profiles/<round>/<name>" in the repository's text files is rewritten to
"profiles/<round>/LOGS.md#<name>", so citations keep resolving.  Longer logs, CSVs, JSON and
directories stay as they are.
"""
from __future__ import annotations

import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    d = os.path.normpath(sys.argv[1])
    max_lines = int(sys.argv[2]) if len(sys.argv) > 2 else 30
    rnd = os.path.basename(d)
    names = sorted(f for f in os.listdir(d) if f.endswith(".log") and os.path.isfile(os.path.join(d, f)))
    fold = []
    for f in names:
        with open(os.path.join(d, f), errors="replace") as fh:
            lines = fh.read().splitlines()
        if len(lines) <= max_lines:
            fold.append((f, lines))
    if not fold:
        print("nothing to fold")
        return
    out = os.path.join(d, "LOGS.md")
    if os.path.exists(out):
        sys.exit(f"{out} exists: fold once per round")
    parts = [f"# Round {rnd[1:]} regression and probe logs\n",
             "Short logs of this round's GPU runs, one section per former file (folded by "
             "`tools/fold_logs.py`).  The table gives each file's last non-empty line: for a bench run "
             "the JSON result, for a test run the pytest summary.\n",
             "| file | lines | last line |", "|---|---|---|"]
    for f, lines in fold:
        last = next((x for x in reversed(lines) if x.strip()), "").strip().replace("|", "\\|")
        if len(last) > 160:
            last = last[:157] + "..."
        parts.append(f"| {f} | {len(lines)} | `{last}` |" if "`" not in last else f"| {f} | {len(lines)} | {last} |")
    parts.append("")
    for f, lines in fold:
        parts += [f"## {f}", "", "```", *lines, "```", ""]
    with open(out, "w") as fh:
        fh.write("\n".join(parts))
    tracked = subprocess.run(["git", "-C", ROOT, "ls-files"], capture_output=True, text=True).stdout.split()
    rel = os.path.relpath(d, ROOT)
    for p in tracked:
        if p.startswith("profiles/") or not p.endswith((".md", ".py", ".hip", ".hpp", ".inl", ".h", ".sh", ".go", ".c")):
            continue
        path = os.path.join(ROOT, p)
        try:
            text = open(path).read()
        except (OSError, UnicodeDecodeError):
            continue
        new = text
        for f, _ in fold:
            new = new.replace(f"{rel}/{f}", f"{rel}/LOGS.md#{f}")
        if new != text:
            with open(path, "w") as fh:
                fh.write(new)
    for f, _ in fold:
        os.remove(os.path.join(d, f))
    print(f"folded {len(fold)} logs into {out}")


if __name__ == "__main__":
    main()
