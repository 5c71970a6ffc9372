"""The oracle (C restatement) against the golden fixtures restating the
reference's own known-answer tests (tests/golden/make_golden.py).  CPU only."""
import numpy as np
import pytest

import oracle as O
from golden_util import assert_array_equal, block_from_rows, encode_inputs, expected_array, load_cases

CASES = load_cases()


@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
def test_oracle_decode_matches_golden(case):
    seg = O.Segment(case["dtypes"])
    data, row_off = block_from_rows(case["rows"])
    if case["expect_error"]:
        with pytest.raises(O.OracleError) as ei:
            O.decode_block(seg, case["proj"], data, row_off)
        assert ei.value.status == 1  # SegmentError("invalid utf8"), utf8.rs:90-92
        assert ei.value.message.startswith("invalid utf8: ")
        return
    got = O.decode_block(seg, case["proj"], data, row_off)
    for p, e in enumerate(case["expected"]):
        assert_array_equal(got[p], expected_array(e), f"{case['name']} col {p}")


@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
def test_oracle_encode_matches_golden(case):
    seg = O.Segment(case["dtypes"])
    n = len(case["rows"])
    blob, row_off = O.encode_batch(seg, encode_inputs(case), n)
    want = case["encode_blobs"] or case["rows"]
    data, off = block_from_rows(want)
    assert np.array_equal(row_off, off)
    assert blob.tobytes() == data.tobytes()


def test_utf8_error_messages_follow_rust_utf8error():
    # core::str::Utf8Error Display, used in utf8.rs:91 format!("invalid utf8: {e}")
    assert O.utf8_valid(b"\xff\xfe\xfd") == (False, 0, 1)
    assert O.utf8_valid(b"ab\xe2\x82") == (False, 2, 0)  # incomplete -> error_len None
    assert O.utf8_valid(b"\xed\xa0\x80") == (False, 0, 1)
    assert O.utf8_valid(b"\xe2\x82\x41") == (False, 0, 2)
    assert O.utf8_valid("δ-unicode😀".encode())[0]


def test_empty_projection_is_arrow_error():
    # RecordBatch::try_new with zero columns fails (src/io/row/read.rs:106-108)
    seg = O.Segment(["float32"])
    with pytest.raises(O.OracleError) as ei:
        O.decode_block(seg, [], np.zeros(0, np.uint8), np.zeros(1, np.uint64))
    assert ei.value.status == 11
