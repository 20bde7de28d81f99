"""Converts the reference's only recorded outputs on the MADS path into a committed fixture
(run in the build container; /root/reference is read-only and absent on the GPU box).

The static N = 5 run of src/FullSimulation.jl (defaults :725-803) wrote
  * Quadrotor_Targets.xlsx — UAV 1's MADS output per MPC step, columns x, y, z
    (src/FullSimulation.jl:370-374 keeps i == 1 only; :655-668 writes it), and
  * Quadrotor_States{i}.xlsx — UAV i's state at the end of each step, columns x, y, z, quaternion
    (:636-652); the next step's MADS starts from it, R = z * tan(FOV/2) (:238-251).
Only x, y, z are kept. Output: tests/golden/quadrotor_run.csv, one line per MPC step:
  tx, ty, tz (UAV 1's target), then x, y, z of UAVs 1..5's end-of-step states.

A second, longer recording sits under src/: src/Quadrotor_Targets.xlsx holds 120 MPC steps of
UAV 1's targets, but its state files come from different runs (src/Quadrotor_States1.xlsx has
40 rows starting near (2, 10), States2/3 120 rows, States4 60), so UAV 1's start of each step is
not recorded for it. Only its targets are kept: tests/golden/quadrotor_run_src.csv, tx, ty, tz
per step — enough to pin the mesh (integer x, y and R = z tan(FOV/2)), not cons3.

Usage: python tests/golden/make_quadrotor_fixture.py
"""
from __future__ import annotations

import os
import re
import zipfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference"


def read_sheet(path: str) -> np.ndarray:
    """Numeric rows of sheet 1 below the header row (inline or shared-string labels skipped)."""
    xml = zipfile.ZipFile(path).read("xl/worksheets/sheet1.xml").decode()
    rows = re.findall(r"<row[^>]*>(.*?)</row>", xml, flags=re.S)
    out = []
    for r in rows[1:]:
        out.append([float(v) for v in re.findall(r"<v>([^<]*)</v>", r)])
    return np.array(out, dtype=np.float64)


def main() -> None:
    T = read_sheet(os.path.join(REF, "Quadrotor_Targets.xlsx"))[:, :3]
    S = [read_sheet(os.path.join(REF, f"Quadrotor_States{i}.xlsx"))[:, :3] for i in range(1, 6)]
    assert all(s.shape == T.shape for s in S), (T.shape, [s.shape for s in S])
    data = np.concatenate([T] + S, axis=1)
    path = os.path.join(HERE, "quadrotor_run.csv")
    with open(path, "w") as f:
        f.write("# src/FullSimulation.jl static run (N=5): UAV 1 target x,y,z; UAV 1..5 end-of-step x,y,z\n")
        for row in data:
            f.write(",".join(repr(float(v)) for v in row) + "\n")
    print(path, data.shape)

    T2 = read_sheet(os.path.join(REF, "src", "Quadrotor_Targets.xlsx"))[:, :3]
    path = os.path.join(HERE, "quadrotor_run_src.csv")
    with open(path, "w") as f:
        f.write("# src/Quadrotor_Targets.xlsx (120 MPC steps): UAV 1 target x,y,z\n")
        for row in T2:
            f.write(",".join(repr(float(v)) for v in row) + "\n")
    print(path, T2.shape)


if __name__ == "__main__":
    main()
