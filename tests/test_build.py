"""build.py's object reuse: a unit's content key covers every unit it #includes (advisor r4),
so an edit to an included unit recompiles its dependants, and nothing else."""
import os
import shutil

import gpdemod_loader

B = gpdemod_loader.load_build()


def test_included_units_are_dependencies():
    assert B.unit_deps("gpd_part6.hip") == ["gpd_part6.hip", "gpd_part2.hip"]
    for u in ("gpd_part9.hip", "gpd_part10.hip", "gpd_part11.hip"):
        assert "gpd_part5.hip" in B.unit_deps(u)
    assert B.unit_deps("gpd_part1.hip") == ["gpd_part1.hip"]
    for u in B.SOURCES:  # every unit a source compiles is itself a listed source
        assert set(B.unit_deps(u)) <= set(B.SOURCES), u


def test_edit_of_an_included_unit_changes_its_dependants_keys(tmp_path, monkeypatch):
    csrc = tmp_path / "csrc"
    shutil.copytree(B.CSRC, csrc)
    monkeypatch.setattr(B, "CSRC", str(csrc))
    before = {u: B.unit_key(u) for u in B.SOURCES}
    with open(csrc / "gpd_part2.hip", "a") as fh:
        fh.write("\n// an edit\n")
    after = {u: B.unit_key(u) for u in B.SOURCES}
    changed = {u for u in B.SOURCES if before[u] != after[u]}
    assert changed == {u for u in B.SOURCES if "gpd_part2.hip" in B.unit_deps(u)}
    assert {"gpd_part2.hip", "gpd_part6.hip"} <= changed
    # a header edit changes every key
    with open(csrc / "gpd_device.hpp", "a") as fh:
        fh.write("\n// an edit\n")
    assert all(B.unit_key(u) != after[u] for u in B.SOURCES)
    # the flags and the build id (unit 0 only) are part of the key
    assert B.unit_key("gpd_part1.hip", ["-DX"]) != B.unit_key("gpd_part1.hip")
    assert B.unit_key("gpd_engine.hip", [], "-DGPD_BUILD_ID=a") != B.unit_key("gpd_engine.hip")
    assert B.unit_key("gpd_part1.hip", [], "-DGPD_BUILD_ID=a") == B.unit_key("gpd_part1.hip")
    assert os.path.exists(os.path.join(B.HERE, "build.py"))
