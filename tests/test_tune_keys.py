"""CPU: the forest's tuning keys agree three ways — the header's list (include/gelly_cc.h, gcc_forest_tune), the keys
gcc_forest_tune accepts (csrc/gelly_cc.hip), and the GPU knob-parity cases (tests/test_gpu_parity.py KNOB_CASES, each
key set away from its default and checked bit-exact on the GPU). A key added in one place only fails here, before a GPU
run."""
import os
import re


ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def code_keys():
    src = open(os.path.join(ROOT, "gelly-streaming_amd", "csrc", "gelly_cc.hip")).read()
    body = src[src.index("int gcc_forest_tune("):]
    body = body[:body.index("\n}\n")]
    keys = set(re.findall(r'k == "([a-z0-9_]+)"', body))
    return keys


def test_header_code_and_gpu_cases_list_the_same_keys():
    from tests.test_gpu_parity import KNOB_CASES, header_tuning_keys

    header = set(header_tuning_keys())
    code = code_keys()
    # fail_absorb is a test hook the header documents apart from the speed knobs
    assert header == code - {"fail_absorb"}, (sorted(header - code), sorted(code - header))
    assert header == set(KNOB_CASES), (sorted(header - set(KNOB_CASES)), sorted(set(KNOB_CASES) - header))
