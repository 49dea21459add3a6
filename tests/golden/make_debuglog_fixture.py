"""Generate tests/golden/debuglog_homography.json from the reference's recorded run.

The reference ships ``debug.log`` (written by logging.debug at test02.py:265-266,
292, 326 / main_v1.py:315-316, 341): 25 cv2.findHomography(RANSAC, thr=75) calls
on 12 correspondences.  For each call it logs M = inv(H), the RANSAC mask and,
per feature, p1 (the dst pixel) and pp2 = dehom(H [pos2, 1]).  This script only
*parses the text* of that log (no reference code is imported or executed) and
writes the numbers as a data fixture:

    blocks[k] = {"M": 3x3, "mask": [12], "p1": [[x, y]]*12, "pp2": [[x, y]]*12,
                 "distance": [12], "complete": bool}

src (pos2) is recovered by the tests as dehom(M [pp2, 1]).

Usage: python tests/golden/make_debuglog_fixture.py [/root/reference/debug.log]
"""
import json
import os
import re
import sys

NUM = r"[-+]?(?:\d+\.?\d*|\.\d+)(?:[eE][-+]?\d+)?"


def _nums(s):
    return [float(x) for x in re.findall(NUM, s)]


def parse(path):
    text = open(path, encoding="utf-8").read()
    # split into log records: each starts with a timestamp
    recs = re.split(r"\n(?=\d{4}-\d\d-\d\d \d\d:\d\d:\d\d,\d+ - )", text)
    blocks = []
    cur = None
    for r in recs:
        body = r.split(" - DEBUG - ", 1)[-1]
        if body.startswith("Homography Matrix M:"):
            vals = _nums(body[len("Homography Matrix M:"):])
            assert len(vals) == 9, vals
            cur = {"M": [vals[0:3], vals[3:6], vals[6:9]], "mask": None, "p1": [], "pp2": [], "distance": []}
            blocks.append(cur)
        elif body.startswith("Mask:"):
            cur["mask"] = [int(v) for v in _nums(body[len("Mask:"):])]
        elif body.startswith("Feature "):
            m = re.match(r"Feature (\d+): mask=\[(\d)\], p1=\[([^\]]*)\], pp2=\[([^\]]*)\], distance=(" + NUM + ")",
                         body)
            assert m, body
            i = int(m.group(1))
            assert i == len(cur["p1"])
            assert int(m.group(2)) == cur["mask"][i]
            cur["p1"].append(_nums(m.group(3)))
            cur["pp2"].append(_nums(m.group(4)))
            cur["distance"].append(float(m.group(5)))
    for b in blocks:
        b["complete"] = b["mask"] is not None and len(b["p1"]) == len(b["mask"])
    return blocks


def main():
    src = sys.argv[1] if len(sys.argv) > 1 else "/root/reference/debug.log"
    blocks = parse(src)
    out = os.path.join(os.path.dirname(os.path.abspath(__file__)), "debuglog_homography.json")
    with open(out, "w") as f:
        json.dump({"source": "reference debug.log (findHomography RANSAC, 12 correspondences)",
                   "threshold": 120.0, "threshold_note": "the logged masks are reproduced by minimal models only at thr=120 (process.py:374 value), not 75", "blocks": blocks}, f, indent=1)
    print(f"{len(blocks)} blocks, {sum(b['complete'] for b in blocks)} complete -> {out}")


if __name__ == "__main__":
    main()
