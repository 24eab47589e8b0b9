"""CPU-side checks of the C-ABI boundary: the library loads, exports every symbol include/flink_window.h
declares, and validates configurations exactly as the reference's constructors do (no GPU needed)."""
import ctypes
import os
import re

import pytest

from flink_amd import _native as N

HEADER = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include", "flink_window.h")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:const\s+)?\w+\s*\*?\s*(fw_\w+)\s*\(", src, flags=re.M)))


def test_header_declares_the_boundary():
    fns = declared_functions()
    for required in ("fw_create", "fw_push_batch", "fw_push_batch_device", "fw_advance_watermark", "fw_destroy",
                     "fw_last_error", "fw_get_stats", "fw_route_device", "fw_key_groups_device"):
        assert required in fns


def test_library_exports_every_declared_symbol():
    L = N.lib()
    fns = declared_functions()
    missing = [f for f in fns if not hasattr(L, f)]
    assert not missing, missing
    # and the Python binding types every one of them
    assert set(fns) == set(N.SIGNATURES), set(fns) ^ set(N.SIGNATURES)


def _create(**kw):
    c = N.FwConfig()
    for k, v in kw.items():
        setattr(c, k, v)
    h = ctypes.c_void_p()
    rc = N.lib().fw_create(ctypes.byref(c), ctypes.byref(h))
    msg = N.lib().fw_last_error(h).decode()
    N.lib().fw_destroy(h)
    return rc, msg


@pytest.mark.parametrize("kw,msg", [
    (dict(assigner=N.FW_TUMBLING, size=100, offset=100), "TumblingEventTimeWindows parameters must satisfy"),
    (dict(assigner=N.FW_TUMBLING, size=-1), "TumblingEventTimeWindows parameters must satisfy"),
    (dict(assigner=N.FW_SLIDING, size=100, slide=10, offset=10), "SlidingEventTimeWindows parameters must"),
    (dict(assigner=N.FW_SLIDING, size=0, slide=10), "SlidingEventTimeWindows parameters must"),
    (dict(assigner=N.FW_SESSION, gap=0), "EventTimeSessionWindows parameters must satisfy"),
    (dict(assigner=N.FW_TUMBLING, size=10, allowed_lateness=-1), "The allowed lateness cannot be negative"),
    (dict(assigner=N.FW_TUMBLING, size=10, max_parallelism=(1 << 15) + 1), "Operator parallelism not within"),
    (dict(assigner=N.FW_TUMBLING, size=10, key_group_start=5, key_group_end=200), "invalid KeyGroupRange"),
    (dict(assigner=N.FW_COUNT, size=0, slide=5, aggregate=N.FW_AGG_FIRST), "count windows need 0 < size"),
    (dict(assigner=N.FW_COUNT, size=10, slide=5), "count windows are offered for countWindow"),
])
def test_create_rejects_invalid_config(kw, msg):
    rc, m = _create(**kw)
    assert rc == N.FW_ERR_ARG
    assert msg in m


def test_kernel_names():
    names = [N.lib().fw_kernel_name(i).decode() for i in range(N.FW_NUM_KERNELS)]
    assert names == ["k_classify_hist", "k_scan", "k_scatter", "k_aggregate", "k_slow", "k_fire", "k_tdigest"]


def test_route_scratch_size_positive():
    assert N.lib().fw_route_scratch_bytes(1 << 20, 8) > 8 * 32 * 4


def test_struct_layouts_match_header(tmp_path):
    # the ctypes mirror against the C compiler's layout of include/flink_window.h, field by field
    import os
    import subprocess
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    fields = [f for f, _ in N.FwConfig._fields_]
    src = tmp_path / "layout.c"
    src.write_text('#include <stdio.h>\n#include <stddef.h>\n#include "flink_window.h"\nint main(void) {\n'
                   '  printf("%zu\\n", sizeof(fw_config));\n' +
                   "".join(f'  printf("%zu\\n", offsetof(fw_config, {f}));\n' for f in fields) + "  return 0;\n}\n")
    exe = tmp_path / "layout"
    subprocess.check_call(["gcc", "-I", os.path.join(root, "include"), str(src), "-o", str(exe)])
    out = [int(x) for x in subprocess.check_output([str(exe)]).split()]
    assert ctypes.sizeof(N.FwConfig) == out[0]
    assert [getattr(N.FwConfig, f).offset for f in fields] == out[1:]
    assert ctypes.sizeof(N.FwRows) == 56
    assert ctypes.sizeof(N.FwStats) == 18 * 8


def test_count_windows_assigner_config():
    from flink_amd import CountWindows
    c = CountWindows.of(10, 5).config()
    assert c == dict(assigner=N.FW_COUNT, size=10, slide=5, count_evict_after=0)
    assert CountWindows.of(4).config()["slide"] == 4  # countWindow(size): tumbling
    assert CountWindows.of(4, 2, evict_after=True).config()["count_evict_after"] == 1
    with pytest.raises(ValueError):
        CountWindows.of(0)


def _list_create(**kw):
    c = N.FwListConfig()
    c.key_group_start = c.key_group_end = -1
    for k, v in kw.items():
        setattr(c, k, v)
    h = ctypes.c_void_p()
    rc = N.lib().fw_list_create(ctypes.byref(c), ctypes.byref(h))
    msg = N.lib().fw_list_last_error(h).decode() if h else ""
    N.lib().fw_list_destroy(h)
    return rc, msg


@pytest.mark.parametrize("kw,msg", [
    (dict(assigner=N.FW_TUMBLING, size=100, offset=100), "TumblingEventTimeWindows parameters must satisfy"),
    (dict(assigner=N.FW_SLIDING, size=100, slide=200), "SlidingEventTimeWindows parameters must satisfy"),
    (dict(assigner=N.FW_TUMBLING, size=10, allowed_lateness=-1), "The allowed lateness cannot be negative"),
    (dict(assigner=N.FW_GLOBAL, trigger=N.FW_TRIGGER_COUNT, trigger_count=0), "CountTrigger count must be in [1, 2^31)"),
    (dict(assigner=N.FW_GLOBAL, evictor=N.FW_EVICT_COUNT, evict_count=-1), "CountEvictor count must be >= 0"),
    (dict(assigner=N.FW_TUMBLING, size=10, key_group_start=5, key_group_end=200), "invalid KeyGroupRange"),
])
def test_list_create_rejects_invalid_config(kw, msg):
    # f4: the window-contents operator validates its configuration before it touches the GPU
    rc, m = _list_create(**kw)
    assert rc == N.FW_ERR_ARG
    assert msg in m


def test_list_struct_layouts_match_header(tmp_path):
    import os
    import subprocess
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    structs = {"fw_list_config": N.FwListConfig, "fw_list_rows": N.FwListRows, "fw_list_elems": N.FwListElems,
               "fw_list_state": N.FwListState}
    body = ""
    for name, cls in structs.items():
        body += f'  printf("%zu\\n", sizeof({name}));\n'
        body += "".join(f'  printf("%zu\\n", offsetof({name}, {f}));\n' for f, _ in cls._fields_)
    src = tmp_path / "layout.c"
    src.write_text('#include <stdio.h>\n#include <stddef.h>\n#include "flink_window.h"\nint main(void) {\n' + body +
                   "  return 0;\n}\n")
    exe = tmp_path / "layout"
    subprocess.check_call(["gcc", "-I", os.path.join(root, "include"), str(src), "-o", str(exe)])
    out = iter(int(x) for x in subprocess.check_output([str(exe)]).split())
    for name, cls in structs.items():
        assert ctypes.sizeof(cls) == next(out), name
        assert [getattr(cls, f).offset for f, _ in cls._fields_] == [next(out) for _ in cls._fields_], name
