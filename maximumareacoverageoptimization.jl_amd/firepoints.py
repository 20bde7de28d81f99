"""FirePoints table: the reference's on-disk fire stream and its CSV form.

The reference writes one XLSX row per fire timestep, each row a flat run of 5-tuples
``[x, y, area, importance, covered]`` (src/DynamicArea.jl:100-108). It reads rows back with
``vec(sheet[row, :])`` + ``filter!(!ismissing, ...)`` and slices groups of 5
(src/CellFunctions.jl:36-41, :63-66). This module converts that table without an XLSX
dependency:
* the reader is stdlib ``zipfile`` + ``xml.etree``;
* the CSV form has one line per timestep and keeps empty timesteps as empty lines, so row t
  stays row t for ``update_POI``'s ``t + 10`` indexing;
* ``#`` lines are comments.

    python -m maximumareacoverageoptimization.jl_amd.firepoints FirePoints.xlsx out.csv
"""
from __future__ import annotations

import sys
import xml.etree.ElementTree as ET
import zipfile

import numpy as np

_NS = {"m": "http://schemas.openxmlformats.org/spreadsheetml/2006/main"}


def _col_index(ref: str) -> int:
    n = 0
    for ch in ref:
        if ch.isalpha():
            n = n * 26 + (ord(ch.upper()) - 64)
        else:
            break
    return n - 1


def read_xlsx(path: str, sheet: int = 1) -> list[np.ndarray]:
    """Rows of the first sheet as (n_i x 5) arrays. Booleans (the "covered" column) become 0/1.
    Missing cells are dropped, as ``filter!(!ismissing, ...)`` drops them."""
    z = zipfile.ZipFile(path)
    root = ET.fromstring(z.read(f"xl/worksheets/sheet{sheet}.xml"))
    shared = []
    if "xl/sharedStrings.xml" in z.namelist():
        sroot = ET.fromstring(z.read("xl/sharedStrings.xml"))
        shared = ["".join(t.text or "" for t in si.iter(f"{{{_NS['m']}}}t"))
                  for si in sroot.findall("m:si", _NS)]
    rows: dict[int, np.ndarray] = {}
    for row in root.find("m:sheetData", _NS).findall("m:row", _NS):
        r = int(row.get("r")) - 1
        cells = {}
        for c in row.findall("m:c", _NS):
            v = c.find("m:v", _NS)
            if v is None:
                continue
            if c.get("t") == "s":
                txt = shared[int(v.text)]
                val = {"true": 1.0, "false": 0.0}.get(txt.strip().lower())
                if val is None:
                    val = float(txt)
            else:
                val = float(v.text)
            cells[_col_index(c.get("r"))] = val
        vals = [cells[i] for i in sorted(cells)]
        if len(vals) % 5:
            raise ValueError(f"row {r + 1}: {len(vals)} values, not a multiple of 5")
        rows[r] = np.array(vals, dtype=np.float64).reshape(-1, 5)
    n = max(rows) + 1 if rows else 0
    return [rows.get(r, np.zeros((0, 5))) for r in range(n)]


def write_csv(rows, path: str, source: str = "") -> str:
    """One line per timestep (empty line = empty timestep), values at full precision."""
    lines = [f"# FirePoints table{(' from ' + source) if source else ''}",
             "# one line per timestep: flat groups [x, y, area, importance, covered]"]
    for a in rows:
        a = np.asarray(a, dtype=np.float64).reshape(-1)
        lines.append(",".join(repr(float(v)) for v in a))
    with open(path, "w") as f:
        f.write("\n".join(lines) + "\n")
    return path


def read_csv(path: str) -> list[np.ndarray]:
    """Inverse of write_csv: a list of (n_i x 5) arrays, empty timesteps kept."""
    rows = []
    with open(path) as f:
        for line in f:
            line = line.rstrip("\n")
            if line.startswith("#"):
                continue
            line = line.strip()
            if not line:
                rows.append(np.zeros((0, 5)))
                continue
            vals = np.array([float(v) for v in line.split(",")], dtype=np.float64)
            if vals.size % 5:
                raise ValueError("FirePoints row length is not a multiple of 5")
            rows.append(vals.reshape(-1, 5))
    return rows


def main(argv=None) -> int:
    argv = sys.argv[1:] if argv is None else argv
    if len(argv) != 2:
        print(__doc__)
        return 2
    rows = read_xlsx(argv[0])
    write_csv(rows, argv[1], source=argv[0])
    print(f"{len(rows)} rows, {sum(r.shape[0] for r in rows)} entries -> {argv[1]}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
