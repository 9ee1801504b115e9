"""The pod jail's policy (native/tools/gpujail.h) against a model of it, on random trees.

``tk8s-gpujail --plan`` prints the Landlock rules the jail would add for a policy without adding
them. For every regular file of a random tree -- with symlinks (inside, dangling, to /), a DRI
root with ``by-path`` links, layers that do not exist -- the access the rules give (the union of
the rules on the file and its ancestors, as Landlock computes it) must be exactly what the most
specific layer says: "/" read-write, --deny none, --read-only read, --allow read-write, and the
render nodes of GPUs not allowed none."""
import json
import os
import subprocess
from pathlib import Path

import pytest
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

from tritonk8ssupervisor_amd.agent.runtime import JAIL

pytestmark = pytest.mark.skipif(not JAIL.exists(), reason="tk8s-gpujail is not built")

RANK = {"none": 0, "r": 1, "rw": 2}
NAMES = ["a", "b", "c", "d"]


def _covers(a: str, b: str) -> bool:
    return a == "/" or b == a or b.startswith(a.rstrip("/") + "/")


@st.composite
def trees(draw):
    """Relative paths: directories, files, symlinks (target: inside, dangling or absolute)."""
    dirs = draw(st.sets(st.lists(st.sampled_from(NAMES), min_size=1, max_size=3).map("/".join), max_size=8))
    files = draw(st.sets(st.tuples(st.sampled_from(sorted(dirs) or [""]), st.sampled_from(["f", "g", "h"])),
                         max_size=10))
    links = draw(st.lists(st.tuples(st.sampled_from(sorted(dirs) or [""]), st.sampled_from(["l", "m"]),
                                    st.sampled_from(["inside", "dangling", "root"])), max_size=3))
    return sorted(dirs), sorted(files), links


@settings(max_examples=40, deadline=None, suppress_health_check=[HealthCheck.function_scoped_fixture])
@given(tree=trees(), data=st.data())
def test_plan_matches_the_most_specific_layer(tmp_path_factory, tree, data):
    root = tmp_path_factory.mktemp("jail").resolve()
    dirs, files, links = tree
    for d in dirs:
        (root / d).mkdir(parents=True, exist_ok=True)
    for d, f in files:
        p = root / d / f
        if not p.exists():
            p.write_text("x")
    link_paths = []
    for d, name, kind in links:
        p = root / d / name
        if p.exists() or p.is_symlink():
            continue
        target = {"inside": str(root / (dirs[0] if dirs else "")), "dangling": str(root / "nowhere"), "root": "/"}[kind]
        os.symlink(target, p)
        link_paths.append(p)
    # a DRI root: render nodes, a card, by-path links to them
    dri = root / "dri"
    (dri / "by-path").mkdir(parents=True)
    for n in ("renderD128", "renderD129", "card0"):
        (dri / n).write_text("")
    os.symlink("../renderD128", dri / "by-path" / "pci-0000:01:00.0-render")
    allow_render = data.draw(st.sets(st.sampled_from([128, 129]), max_size=2))

    candidates = [root / d for d in dirs] + [root / d / f for d, f in files] + link_paths + [root / "missing"]
    pick = lambda: data.draw(st.lists(st.sampled_from(candidates), max_size=3))  # noqa: E731
    deny, ro, allow = pick(), pick(), pick()
    argv = [str(JAIL), "--dri-root", str(dri), "--kfd-root", str(root / "no-kfd")]
    for m in sorted(allow_render):
        argv += ["--allow-render", str(m)]
    for opt, paths in (("--deny", deny), ("--read-only", ro), ("--allow", allow)):
        for p in paths:
            argv += [opt, str(p)]
    r = subprocess.run(argv + ["--plan"], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr
    rules = [json.loads(line) for line in r.stdout.splitlines()]

    # the model: most specific layer; later options win for the same path (deny < read-only < allow)
    layers = {"/": "rw"}
    for n in ("renderD128", "renderD129", "card0"):
        if not (n.startswith("renderD") and int(n[7:]) in allow_render):
            layers[str(dri / n)] = "none"
    for paths, acc in ((deny, "none"), (ro, "r"), (allow, "rw")):
        for p in paths:
            if os.path.exists(p) and not (acc == "none" and os.path.realpath(p) == "/"):  # "/" is never denied
                layers[os.path.realpath(p)] = acc

    def expected(path: str) -> str:
        best = max((lp for lp in layers if _covers(lp, path)), key=len)
        return layers[best]

    def granted(path: str) -> str:
        got = [x["access"] for x in rules if _covers(x["path"], path)]
        return max(got, key=RANK.get, default="none")

    checked = 0
    for p in root.rglob("*"):
        if p.is_symlink() or not p.is_file():
            continue
        rp = os.path.realpath(p)
        assert granted(rp) == expected(rp), (rp, layers, [x for x in rules if str(root) in x["path"]])
        checked += 1
    assert checked >= 3  # the DRI nodes at least
