"""The C-ABI boundary (CPU-only checks; no compute call needs a GPU here).

* libvsim_hip.so loads and exports every function include/*.h declares;
* the ggml ABI mirror (include/ggml_abi.h) has the reference's layout;
* the host-built fp16 tables the device uses equal the reference's tables.
"""
import os
import re
import subprocess
import tempfile

import numpy as np
import pytest

from vsim_amd import hip

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
REF = "/root/reference"


def declared_functions():
    names = set()
    for h in ("vsim_hip.h",):
        src = open(os.path.join(ROOT, "include", h)).read()
        src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
        for m in re.finditer(r"^\s*(?:const\s+)?[A-Za-z_][\w\s\*]*?\b([A-Za-z_]\w*)\s*\(", src, flags=re.M):
            name = m.group(1)
            if name not in ("if", "sizeof", "defined"):
                names.add(name)
    return names


def exported_symbols():
    out = subprocess.run(["nm", "-D", "--defined-only", hip.LIB_PATH], capture_output=True, text=True, check=True)
    return {ln.split()[-1] for ln in out.stdout.splitlines() if ln.strip()}


def test_library_loads():
    L = hip.lib()
    assert L.vsim_q4_bytes(4096, 4096) == 4096 * 4096 // 32 * 20


def test_every_declared_symbol_is_exported():
    decl = declared_functions()
    assert "imax_ggml_compute_forward_mul_mat_q4_0_f32" in decl and "init_xmax" in decl
    missing = decl - exported_symbols()
    assert not missing, f"declared in include/vsim_hip.h but not exported: {sorted(missing)}"
    assert set(hip.EXPORTS) <= exported_symbols()


def _offsets_program(header_include: str) -> str:
    fields = ["type", "n_dims", "ne", "nb", "op", "is_param", "grad", "src0", "src1", "opt", "n_tasks",
              "perf_runs", "perf_cycles", "perf_time_us", "data", "padding"]
    lines = [f'printf("{f} %zu\\n", offsetof(struct ggml_tensor, {f}));' for f in fields]
    return f"""
#include <stddef.h>
#include <stdio.h>
{header_include}
int main(void) {{
  {' '.join(lines)}
  printf("sizeof %zu\\n", sizeof(struct ggml_tensor));
  printf("GGML_OP_MUL_MAT %d\\nGGML_OP_GPTNEOX_ROPE %d\\nGGML_OP_COUNT %d\\n", (int)GGML_OP_MUL_MAT,
         (int)GGML_OP_GPTNEOX_ROPE, (int)GGML_OP_COUNT);
  return 0;
}}
"""


def _run_c(src: str, incdir: str) -> str:
    d = tempfile.mkdtemp()
    c = os.path.join(d, "t.c")
    open(c, "w").write(src)
    exe = os.path.join(d, "t")
    subprocess.run(["gcc", "-I", incdir, c, "-o", exe], check=True)
    return subprocess.run([exe], capture_output=True, text=True, check=True).stdout


def test_ggml_abi_layout():
    mine = _run_c(_offsets_program('#include "ggml_abi.h"'), os.path.join(ROOT, "include"))
    assert "sizeof" in mine
    if not os.path.exists(os.path.join(REF, "ggml.h")):
        pytest.skip("reference headers not present on this machine")
    ref = _run_c(_offsets_program('#include <pthread.h>\n#include <signal.h>\n#include "ggml.h"'), REF)
    assert mine == ref


def _cgraph_program(header_include: str) -> str:
    fields = ["n_nodes", "n_leafs", "n_threads", "work_size", "work", "nodes", "grads", "leafs", "perf_runs",
              "perf_cycles", "perf_time_us"]
    lines = [f'printf("{f} %zu\\n", offsetof(struct ggml_cgraph, {f}));' for f in fields]
    return f"""
#include <stddef.h>
#include <stdio.h>
{header_include}
int main(void) {{
  {' '.join(lines)}
  printf("sizeof %zu\\n", sizeof(struct ggml_cgraph));
  return 0;
}}
"""


def test_ggml_cgraph_layout():
    """vsim_graph_compute reads the reference's struct ggml_cgraph (ggml.h:308-324)."""
    mine = _run_c(_cgraph_program('#include "ggml_abi.h"'), os.path.join(ROOT, "include"))
    assert "sizeof" in mine
    if not os.path.exists(os.path.join(REF, "ggml.h")):
        pytest.skip("reference headers not present on this machine")
    ref = _run_c(_cgraph_program('#include <pthread.h>\n#include <signal.h>\n#include "ggml.h"'), REF)
    assert mine == ref


def test_ggml_context_head_layout():
    """vsim_graph_compute reads mem_size / mem_buffer, the first fields of ggml.c's private
    struct ggml_context (ggml.c:1022-1024): compile the reference's ggml.c with static
    assertions on those offsets (compile only, nothing runs)."""
    if not os.path.exists(os.path.join(REF, "ggml.c")):
        pytest.skip("reference sources not present on this machine")
    d = tempfile.mkdtemp()
    c = os.path.join(d, "t.c")
    open(c, "w").write(f'#include "{REF}/ggml.c"\n'
                       "_Static_assert(offsetof(struct ggml_context, mem_size) == 0, \"mem_size\");\n"
                       "_Static_assert(offsetof(struct ggml_context, mem_buffer) == sizeof(size_t), \"mem_buffer\");\n")
    subprocess.run(["gcc", "-I", REF, "-pthread", "-fcommon", "-w", "-c", c, "-o", os.path.join(d, "t.o")],
                   check=True)


def test_fp16_tables_match_reference():
    import oracle_py as O
    e_ref, g_ref = O.tables()
    e = np.zeros(65536, np.uint16)
    g = np.zeros(65536, np.uint16)
    hip.check(hip.lib().vsim_op_tables(hip.ptr(e), hip.ptr(g)), "tables")
    assert np.array_equal(e, e_ref)
    assert np.array_equal(g, g_ref)


def test_ctypes_ggml_mirror_layout():
    """vsim_amd.hip.GgmlTensor (the Python callers' mirror) has include/ggml_abi.h's layout."""
    mine = _run_c(_offsets_program('#include "ggml_abi.h"'), os.path.join(ROOT, "include"))
    want = dict(ln.split()[:2] for ln in mine.splitlines() if not ln.startswith("GGML_"))
    import ctypes
    for name, _ in hip.GgmlTensor._fields_:
        assert getattr(hip.GgmlTensor, name).offset == int(want[name]), name
    assert ctypes.sizeof(hip.GgmlTensor) == int(want["sizeof"])
