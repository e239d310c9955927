"""The shipped library holds no packed-FP32 instruction that feeds the low lane from src1's / src2's high register
(the gfx950 form that dropped dgamma rows in round 5: tools/isa_audit.py).  CPU only: the
gfx950 code objects are read out of libtagan_hip.so and disassembled with llvm-objdump."""
import glob
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import isa_audit  # noqa: E402

PKG = os.path.join(ROOT, "temporal-asymmetric-graph-attention-network_amd")


def test_classifier_on_the_round5_encodings():
    bad = ["v_pk_mul_f32 v[96:97], v[94:95], v[180:181] op_sel:[0,1] op_sel_hi:[1,0]",
           "v_pk_fma_f32 v[16:17], v[20:21], v[28:29], v[16:17] op_sel:[0,1,0] op_sel_hi:[1,0,1]",
           "v_pk_add_f32 v[16:17], v[14:15], v[14:15] op_sel:[0,1] op_sel_hi:[1,0]",
           "v_pk_fma_f32 v[2:3], v[4:5], v[6:7], v[8:9] op_sel:[0,0,1]"]
    good = ["v_pk_mul_f32 v[96:97], v[180:181], v[94:95] op_sel:[1,0] op_sel_hi:[0,1]",   # the commuted form
            "v_pk_mul_f32 v[0:1], v[2:3], v[4:5]",
            "v_pk_fma_f32 v[0:1], v[2:3], v[4:5], v[6:7] op_sel_hi:[0,1,1]",
            "v_pk_mul_f32 v[0:1], v[2:3], s[4:5] op_sel_hi:[1,0]",
            "v_mul_f32_e32 v96, v94, v181"]
    assert all(isa_audit.forbidden(x) for x in bad)
    assert not any(isa_audit.forbidden(x) for x in good)


@pytest.mark.parametrize("name", ["libtagan_hip.so", "libtagan_hip_debug.so"])
def test_library_has_no_src1_high_packed_fp32(name):
    path = os.path.join(PKG, name)
    if not os.path.exists(path):
        pytest.skip(name + " not built")
    findings, census = isa_audit.audit(path)
    assert sum(census.values()) > 0          # the audit saw the code (packed FP32 stays on in the other files)
    assert not findings, findings[:5]
