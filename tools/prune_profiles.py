"""List (or delete) profiles/ files that nothing cites.

  python tools/prune_profiles.py          # dry run: counts and the files it would remove
  python tools/prune_profiles.py --apply  # git rm them

A file is kept when DESIGN.md, README.md, INTEGRATION.md, profiles/README.md, bench.py or a
test names it -- literally, or through a brace / glob pattern such as
profiles/lat_r05n_q{0,8192}_*.txt -- or when it belongs to the current round (--keep-tag).
Old rounds' raw logs stay in git history.
"""
import fnmatch
import itertools
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CITERS = ["DESIGN.md", "README.md", "INTEGRATION.md", os.path.join("profiles", "README.md"), "bench.py"]


def brace_expand(p):
    m = re.search(r"\{([^{}]*)\}", p)
    if not m:
        return [p]
    out = []
    for alt in m.group(1).split(","):
        out += brace_expand(p[:m.start()] + alt + p[m.end():])
    return out


def main():
    keep_tags = [a.split("=", 1)[1] for a in sys.argv[1:] if a.startswith("--keep-tag=")] or ["r06"]
    files = sorted(f for f in os.listdir(os.path.join(ROOT, "profiles")) if f != "README.md")
    text = ""
    for c in CITERS:
        p = os.path.join(ROOT, c)
        if os.path.exists(p):
            text += open(p).read() + "\n"
    for t in os.listdir(os.path.join(ROOT, "tests")):
        if t.endswith(".py"):
            text += open(os.path.join(ROOT, "tests", t)).read() + "\n"
    # every token that looks like a profile file name or pattern
    toks = set(re.findall(r"[A-Za-z0-9_.{},*\-]+\.(?:json|md|txt|log|csv)", text))
    toks |= set(re.findall(r"[A-Za-z0-9_{},*\-]+_\*", text))
    pats = set()
    for t in toks:
        for e in brace_expand(t):
            pats.add(e.split("/")[-1])
    keep = set()
    for f in files:
        if any(t in f for t in keep_tags):
            keep.add(f)
            continue
        for p in pats:
            if f == p or fnmatch.fnmatch(f, p) or (p.endswith("_*") and fnmatch.fnmatch(f, p + "*")):
                keep.add(f)
                break
        else:
            # "pmc_r05zzzzz_*" style prefixes cited without the suffix
            stem = f.split(".")[0]
            if re.search(re.escape(stem) + r"\b", text):
                keep.add(f)
    drop = [f for f in files if f not in keep]
    # the newest PMC summary is read by bench.py at run time: never dropped
    pmc = sorted(f for f in files if f.startswith("pmc_") and f.endswith("_counters.json"))
    if pmc:
        drop = [f for f in drop if f != pmc[-1]]
    print("profiles: %d files, keep %d, drop %d" % (len(files), len(files) - len(drop), len(drop)))
    if "--apply" in sys.argv:
        for chunk in (drop[i:i + 100] for i in range(0, len(drop), 100)):
            subprocess.run(["git", "rm", "-q", "--"] + [os.path.join("profiles", f) for f in chunk], cwd=ROOT,
                           check=True)
    else:
        for f in drop:
            print("  drop", f)


if __name__ == "__main__":
    main()
