#!/bin/bash
# Build provenance: extract the committed tree (git archive HEAD: no built files), run build() there from
# scratch, and compare the fresh library's embedded source sha256 with the in-tree library's.
set -eo pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
D=$(mktemp -d /tmp/grid_clean_build.XXXX)
git -C "$ROOT" archive HEAD | tar -x -C "$D"
test ! -e "$D/grid_amd/_lib"
t0=$(date +%s)
(cd "$D" && python -c "import __graft_entry__ as g; g.build()") > "$D.log" 2>&1
t1=$(date +%s)
python - "$ROOT" "$D" $((t1 - t0)) "$(git -C "$ROOT" rev-parse HEAD)" <<'PY'
import json, subprocess, sys
root, d, secs, rev = sys.argv[1:]
def info(tree):
    code = "import sys; sys.path.insert(0, %r); from grid_amd import _abi; print(__import__('json').dumps(_abi.build_info()))" % tree
    return json.loads(subprocess.check_output([sys.executable, "-c", code], text=True))
fresh, shipped = info(d), info(root)
print(json.dumps({"commit": rev, "clean_build_s": int(secs), "fresh_library": fresh, "in_tree_library": shipped,
                  "same_sources": fresh["src_sha256"] == shipped["src_sha256"]}, indent=1))
PY
rm -rf "$D" "$D.log"
