"""Housekeeping: every tracked file under profiles/ is named — itself, or a directory it sits in — by a
round's INDEX.md, profiles/README.md or the design docs, so that the measured evidence stays what the
docs cite (prune profiles/ to what the indexes cite).  No GPU."""
import os
import re
import subprocess

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_every_profile_file_is_cited():
    files = subprocess.run(["git", "ls-files", "profiles"], cwd=REPO, capture_output=True, text=True,
                           check=True).stdout.split()
    if not files:  # not a git checkout (the GPU box's snapshot has no .git)
        return
    docs = ""
    for p in ["DESIGN.md", "DESIGN_LOG.md", "README.md", "profiles/README.md"] + \
             [f for f in files if f.endswith("INDEX.md")]:
        path = os.path.join(REPO, p)
        if os.path.exists(path):
            docs += open(path).read()
    missing = []
    for f in files:
        rel = f[len("profiles/"):]
        parts = rel.split("/")
        name = parts[-1]
        cited = name in docs or rel in docs or name in ("README.md", "INDEX.md")
        for k in range(1, len(parts)):
            d = "/".join(parts[:k])
            cited = cited or (d + "/") in docs or ("`" + d + "`") in docs
        if not cited:  # brace patterns: bench_{cornell,blob}.json, ..._{a,b}_pmc.json
            for m in re.finditer(r"`([^`]*\{[^`]*\}[^`]*)`", docs):
                pat = re.escape(m.group(1)).replace(r"\{", "(").replace(r"\}", ")").replace(",", "|")
                pat = pat.replace(r"\|", "|").replace(r"\(", "(").replace(r"\)", ")")
                try:
                    if re.search(pat + "$", rel):
                        cited = True
                        break
                except re.error:
                    continue
        if not cited:
            missing.append(f)
    assert not missing, f"{len(missing)} profile files no index names: {missing[:10]}"
