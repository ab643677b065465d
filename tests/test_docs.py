"""The evidence the documents cite exists in the tree: every backticked
repository path in DESIGN.md, README.md, INTEGRATION.md and tools/README.md
(profiles, tools, tests, sources) names a file that is there, except the
scripts the documents themselves record as removed and build outputs
(git-ignored, made by __graft_entry__.build())."""
import os
import re

from conftest import ROOT

DOCS = ["DESIGN.md", "README.md", "INTEGRATION.md", os.path.join("tools", "README.md")]
REMOVED = {"tools/diag_variants.sh"}  # removed in round 4, named for the record
PATH = re.compile(r"`((?:profiles|tools|tests|host|oracle|memo_amd|include)/[A-Za-z0-9_./-]+)`")


def test_cited_paths_exist():
    missing = []
    for doc in DOCS:
        with open(os.path.join(ROOT, doc)) as f:
            text = f.read()
        for p in PATH.findall(text):
            p = p.rstrip(".,")
            built = any(d in p.split("/") for d in ("_lib", "_build", "_bin", "_ref"))
            if p not in REMOVED and not built and not os.path.exists(os.path.join(ROOT, p)):
                missing.append((doc, p))
    assert not missing, missing
