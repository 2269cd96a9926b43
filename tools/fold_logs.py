"""Fold a round's short regression logs into one file (profiles/<round>/LOGS.md).

usage: python tools/fold_logs.py profiles/r03 [max_lines] [--append] [--trim H,T] [--drop GLOB ...]

Every *.log directly in the directory with at most max_lines (default 30) lines becomes one
section of LOGS.md, headed by its old file name, under a summary table (file, lines, its last
non-empty line -- for a bench or test log, the result line).  The folded files are removed and
every reference to "profiles/<round>/<name>" in the repository's text files is rewritten to
"profiles/<round>/LOGS.md#<name>", so citations keep resolving.  Longer logs, CSVs, JSON and
directories stay as they are.
  --append   add to an existing LOGS.md (a second fold in the same round)
  --trim H,T keep only the first H and last T lines of a folded log longer than H + T (a pytest
             -v listing's middle; the whole file stays in git history at the current commit)
  --drop G   delete the logs matching glob G instead of folding them (closed investigations)
"""
from __future__ import annotations

import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    import argparse
    import fnmatch
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("max_lines", nargs="?", type=int, default=30)
    ap.add_argument("--append", action="store_true")
    ap.add_argument("--trim", default="")
    ap.add_argument("--drop", action="append", default=[])
    a = ap.parse_args()
    d = os.path.normpath(a.dir)
    max_lines = a.max_lines
    rnd = os.path.basename(d)
    head = subprocess.run(["git", "-C", ROOT, "rev-parse", "--short", "HEAD"], capture_output=True,
                          text=True).stdout.strip()
    names = sorted(f for f in os.listdir(d) if os.path.isfile(os.path.join(d, f))
                   and (f.endswith(".log") or any(fnmatch.fnmatch(f, g) for g in a.drop)))
    for f in names:
        if any(fnmatch.fnmatch(f, g) for g in a.drop):
            os.remove(os.path.join(d, f))
            print(f"dropped {f}")
    names = [f for f in names if os.path.exists(os.path.join(d, f))]
    keep_h, keep_t = (int(x) for x in a.trim.split(",")) if a.trim else (0, 0)
    fold = []
    for f in names:
        with open(os.path.join(d, f), errors="replace") as fh:
            lines = fh.read().splitlines()
        if len(lines) <= max_lines:
            n = len(lines)
            if a.trim and n > keep_h + keep_t:
                lines = lines[:keep_h] + [f"[... {n - keep_h - keep_t} lines elided: the whole file is "
                                          f"profiles/{rnd}/{f} at commit {head} ...]"] + lines[n - keep_t:]
            fold.append((f, lines))
    if not fold:
        print("nothing to fold")
        return
    out = os.path.join(d, "LOGS.md")
    if os.path.exists(out) and not a.append:
        sys.exit(f"{out} exists: fold once per round (or --append)")
    if a.append:
        with open(out) as fh:
            parts = [fh.read().rstrip("\n"), "", f"## Folded later in round {rnd[1:]}", "",
                     "| file | lines | last line |", "|---|---|---|"]
    else:
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
