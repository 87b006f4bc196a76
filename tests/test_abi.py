"""CPU tests of the drop-in boundary (include/stomp_engine.h): the HIP library
loads without a GPU, exports every declared symbol, the ctypes mirror of every
struct has the C layout, and argument validation fails loudly before any device
call.  No compute runs here (no GPU in this container)."""
import ctypes as C
import os
import re
import subprocess

import numpy as np
import pytest

from stomp_motion_planner_icra2011_amd import engine as eng
from stomp_motion_planner_icra2011_amd import problem as pb

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "stomp_engine.h")
ORACLE_HEADER = os.path.join(ROOT, "oracle", "stomp_oracle.h")


def declared_functions(path):
    text = open(path).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"^[A-Za-z_][\w \*]*?\b((?:stomp|so)_\w+)\s*\(", text, flags=re.M)))


def test_header_declares_the_binding_list():
    assert declared_functions(HEADER) == sorted(eng.EXPORTED)


def test_engine_library_exports_every_symbol():
    lib = eng.load_library()
    missing = [f for f in declared_functions(HEADER) if not hasattr(lib, f)]
    assert not missing, missing


def test_library_carries_the_checkout_source_hash(tmp_path):
    # the product library is bound to its sources: the hash compiled into it is the checkout's, and
    # a library built from other sources is refused by the binding
    from stomp_motion_planner_icra2011_amd import _build
    lib = eng.load_library()
    assert lib.stomp_engine_source_hash().decode() == _build.source_hash()
    assert _build.embedded_hash(_build.LIB) == _build.source_hash()
    stale = tmp_path / "libstomp_engine.so"
    data = open(_build.LIB, "rb").read().replace(b"STOMP_SOURCE_HASH=" + _build.source_hash().encode(),
                                                 b"STOMP_SOURCE_HASH=0123456789abcdef")
    stale.write_bytes(data)
    assert _build.embedded_hash(str(stale)) == "0123456789abcdef"
    import subprocess, sys, textwrap
    code = textwrap.dedent(f"""
        import sys; sys.path.insert(0, {repr(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))})
        from stomp_motion_planner_icra2011_amd import engine as eng
        eng._LIB_PATH = {repr(str(stale))}
        try:
            eng.load_library()
        except RuntimeError as ex:
            print("refused:", ex)
    """)
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, env={**os.environ, "STOMP_ENGINE_LIB": ""})
    assert "refused: stale STOMP engine library" in out.stdout, out.stdout + out.stderr


def test_oracle_library_exports_every_symbol():
    from oracle import pyoracle as po
    lib = po.lib()
    missing = [f for f in declared_functions(ORACLE_HEADER) if not hasattr(lib, f)]
    assert not missing, missing


def test_struct_layouts_match_c(tmp_path):
    structs = {"stomp_segment": eng.stomp_segment, "stomp_sphere": eng.stomp_sphere,
               "stomp_joint": eng.stomp_joint, "stomp_grid": eng.stomp_grid,
               "stomp_engine_desc": eng.stomp_engine_desc, "stomp_iter_out": eng.stomp_iter_out,
               "stomp_inertia": eng.stomp_inertia, "stomp_orientation_constraint": eng.stomp_orientation_constraint,
               "stomp_stats": eng.stomp_stats}
    lines = ['#include <stdio.h>', '#include <stddef.h>', '#include "stomp_engine.h"', "int main(void){"]
    for name, cls in structs.items():
        lines.append(f'printf("{name} %zu\\n", sizeof({name}));')
        for field, _ in cls._fields_:
            lines.append(f'printf("{name}.{field} %zu\\n", offsetof({name}, {field}));')
    lines.append("return 0;}")
    src = tmp_path / "layout.c"
    src.write_text("\n".join(lines))
    exe = tmp_path / "layout"
    subprocess.check_call(["gcc", "-std=c99", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)])
    out = dict(l.rsplit(" ", 1) for l in subprocess.check_output([str(exe)], text=True).splitlines())
    for name, cls in structs.items():
        assert int(out[name]) == C.sizeof(cls), name
        for field, _ in cls._fields_:
            assert int(out[f"{name}.{field}"]) == getattr(cls, field).offset, f"{name}.{field}"


def test_header_compiles_as_c_and_cpp(tmp_path):
    src = tmp_path / "h.c"
    src.write_text('#include "stomp_engine.h"\nint main(void){return STOMP_ENGINE_ABI_VERSION - 1;}\n')
    for compiler, flag in (("gcc", "-std=c99"), ("g++", "-std=c++11")):
        subprocess.check_call([compiler, flag, "-x", "c" if compiler == "gcc" else "c++", "-Wall", "-Werror",
                               "-I", os.path.join(ROOT, "include"), str(src), "-o", str(tmp_path / "h")])


@pytest.mark.parametrize("kw,code,msg", [
    (dict(num_rollouts=10, num_reused_rollouts=10), -1, "strictly less"),
    (dict(dof=14, num_rollouts=10, num_reused_rollouts=0, torque_cost_weight=0.001), -3, "group joints"),
    (dict(num_rollouts=10, num_reused_rollouts=0, torque_cost_weight=0.001, torque_tip="torso_lift_link"), -3,
     "group joints"),
])
def test_create_validates_before_touching_the_device(kw, code, msg):
    tip = kw.pop("torque_tip", None)
    p = pb.make_problem(grid_n=16, **kw)
    if tip:
        p.torque_tip = tip
    with pytest.raises(RuntimeError) as ei:
        eng.Engine(p)
    assert f"error {code}" in str(ei.value) and msg in str(ei.value)


def test_multi_rank_requires_whole_sum_blocks():
    p = pb.make_problem(grid_n=16, num_rollouts=96, num_reused_rollouts=0)
    with pytest.raises(RuntimeError) as ei:
        eng.Engine(p, rank=0, world_size=2, comm_id=b"\0" * 128)
    assert "multiple of 64" in str(ei.value)


def test_abi_version_mismatch_rejected():
    lib = eng.load_library()
    d = eng.stomp_engine_desc()
    d.abi_version = 999
    h = C.c_void_p()
    assert lib.stomp_engine_create(C.byref(d), C.byref(h)) == -1
    assert b"abi_version" in lib.stomp_last_error()
    assert not h.value


@pytest.mark.parametrize("rank,comm,msg", [(0, None, "needs a comm_id"), (2, b"\0" * 128, "outside [0, world_size 2)"),
                                           (-1, b"\0" * 128, "outside")])
def test_multi_rank_arguments_checked(rank, comm, msg):
    p = pb.make_problem(grid_n=16, num_rollouts=128, num_reused_rollouts=0)
    with pytest.raises(RuntimeError) as ei:
        eng.Engine(p, rank=rank, world_size=2, comm_id=comm)
    assert msg in str(ei.value)


def test_local_group_ids_are_distinct():
    a, b = eng.comm_local_id(2), eng.comm_local_id(2)
    assert a[:8] == b"STOMPLOC" and b[:8] == b"STOMPLOC" and a != b and len(a) == 128


def test_float_field_rejected():
    # ABI v4 holds the field as integer squared cell distances: a field in metres is refused, not
    # truncated to "everything in collision" 
    p = pb.make_problem(grid_n=16, num_rollouts=10, num_reused_rollouts=0)
    p.sdf = np.full((16, 16, 16), 0.35, np.float32)
    with pytest.raises(TypeError, match="integer squared cell distances"):
        eng.Engine(p)
    p.sdf = np.full((16, 16, 16), 70000, np.int64)
    with pytest.raises(ValueError, match="65535"):
        eng.Engine(p)


def test_shard_decide_rule():
    # the K-sharded decomposition from measured times (us): gather posts one all-gather of the
    # state rows, partials three dependent collectives (stomp_shard_decide)
    assert eng.shard_decide(51.4, 42.7, 20.0, 25.0, 20.0) == "gather"      # RCCL-like latencies
    assert eng.shard_decide(51.4, 42.7, 1.0, 2.0, 1.0) == "partials"       # collectives cheaper than the compute gap
    assert eng.shard_decide(40.0, 40.0, 0.0, 0.0, 0.0) == "gather"         # ties: one collective
