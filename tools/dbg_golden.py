"""Debug helper: decode one golden case on the GPU and print every buffer."""
import json, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
from golden_util import block_from_rows, load_cases  # noqa
from murr_amd.device import Context, DeviceBlock, decode_blocks, download_array
from murr_amd.schema import SegmentSchema, DTypeName as D

name = sys.argv[1] if len(sys.argv) > 1 else "row_with_nulls"
case = [c for c in load_cases() if c["name"] == name][0]
seg = SegmentSchema([(f"c{i}", D.parse(d)) for i, d in enumerate(case["dtypes"])])
data, off = block_from_rows(case["rows"])
with Context(0) as ctx:
    for proj in ([0, 1], [1, 0], [0], [1], [0, 0, 1]):
        outs = decode_blocks(ctx, seg, proj, [DeviceBlock.upload(ctx, data, off)])
        for p, c in enumerate(proj):
            a = download_array(ctx, outs.array(0, p), int(seg.columns[c].dtype), len(off) - 1)
            print(proj, p, {k: (v.hex() if isinstance(v, (bytes, bytearray)) else v) for k, v in a.items()})
