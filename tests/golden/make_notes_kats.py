"""Transcribes the OpenCV match lists the reference's author logged from real
runs into tests/golden/notes_match_lists.json (data only: distance, trainIdx,
queryIdx of each logged top-10 list, with its source line).

Source: /root/reference/scripts/back_up_files/frame_extraction_notes.txt
(run in this container; the fixture travels, the reference does not).
Lists printed after the reference's stable sort (visual_odometry_v3.py:221)
are "sorted"; the ones printed "BEFORE ADDING THE SORT" are BFMatcher's raw
output ("raw").  Also records interesting_phenomenon.txt:7 (both keypoint
lists of a default ORB_create() run held 500 entries)."""
import ast
import json
import os
import re

REF = "/root/reference/scripts/back_up_files"


def main():
    lines = open(os.path.join(REF, "frame_extraction_notes.txt")).read().split("\n")
    lists = []
    i = 0
    while i < len(lines):
        if "Here are the top 10 matches:" in lines[i]:
            start = i + 1
            text = lines[i].split("matches:", 1)[1]
            j = i
            while text.count("[") == 0 or text.count("[") != text.count("]"):
                j += 1
                text += lines[j]
            ms = ast.literal_eval(text.strip())
            lists.append({"line": start, "matches": [[m["distance"], m["trainIdx"], m["queryIdx"]] for m in ms]})
            i = j
        i += 1
    # the two lists printed "BEFORE ADDING THE SORT MATCHES BY LAMBDA DISTANCE" come after that header
    before = next(k for k, l in enumerate(lines) if "BEFORE ADDING THE SORT" in l) + 1
    for L in lists:
        L["kind"] = "raw" if L["line"] > before else "sorted"
    ph = open(os.path.join(REF, "interesting_phenomenon.txt")).read().split("\n")
    k = next(n for n, l in enumerate(ph) if re.search(r"LIST \d+, \d+", l))
    counts = [int(x) for x in re.findall(r"\d+", ph[k])]
    out = {"source": "scripts/back_up_files/frame_extraction_notes.txt (matches: [distance, trainIdx, queryIdx])",
           "lists": lists,
           "keypoint_counts": {"source": f"scripts/back_up_files/interesting_phenomenon.txt:{k + 1}",
                               "counts": counts, "nfeatures": 500}}
    json.dump(out, open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "notes_match_lists.json"), "w"),
              indent=1)


if __name__ == "__main__":
    main()
