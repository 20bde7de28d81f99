"""Mirror of src/DynamicArea.jl: the cellular-automaton forest fire that produces the fire-point
stream (config 5), running on the GPU (``mac_fire_*``, csrc/fire.hip).

The module constants are the reference's (:6-21, :47-48). Grid cell (i, j) is 1-based, with i
the row (x index) and j the column (y index), as the reference indexes ``grid[i, j]``. Points
are 5-tuples ``[x, y, area, importance, covered]``, pushed one per igniting neighbour (:65).
The reference's ``rand()`` is unseeded. Here the draws are a counter-based hash of
(seed, step, cell, neighbour), identical on the tests' CPU restatement, so runs are
reproducible and parity-testable.
"""
from __future__ import annotations

import math

import numpy as np

from ._lib import Context, Fire

EMPTY, TREE, FIRE = 0, 1, 2                    # :17
dx = 5                                         # :6
dy = 5                                         # :7
X = 500                                        # :9
Y = 500                                        # :10
x_start1, x_start2 = 200, 300                  # :11-12
y_start1, y_start2 = 345, 355                  # :13-14
num_iterations = 100                           # :18
forest_density = 0.7                           # :20
prob_spread = 0.5                              # :21
wind_speed = 4                                 # :47
wind_direction = math.radians(270)             # :48
SEED = 20250216


def _jround(v: float) -> int:
    """Julia's round (ties to even); Python's round does the same."""
    return int(round(v))


class DynamicArea:
    """One fire simulation (grid state on the GPU)."""

    def __init__(self, X=X, Y=Y, dx=dx, dy=dy, x_start1=x_start1, x_start2=x_start2,
                 y_start1=y_start1, y_start2=y_start2, forest_density=forest_density,
                 prob_spread=prob_spread, wind_speed=wind_speed, wind_direction=wind_direction,
                 seed=SEED, device: int = 0):
        self.dx, self.dy = dx, dy
        self.grid_size = (_jround(X / dx), _jround(Y / dy))                       # :19
        self.ignition = (_jround(x_start1 / dx), _jround(x_start2 / dx),          # :35
                         _jround(y_start1 / dy), _jround(y_start2 / dy))
        self.fire = Fire(self.grid_size[0], self.grid_size[1], float(dx), float(dy),
                         forest_density, prob_spread, float(wind_speed), wind_direction,
                         self.ignition, seed, device)
        self.export_data = [self.initial_points()]                                # :43

    def initial_points(self) -> np.ndarray:
        """:37-42, y outer and x inner."""
        return self.fire.initial_points()

    def update_grid(self, append_to: Context | None = None) -> np.ndarray:
        """:52-72. Returns this step's points (n, 5). They are appended to append_to's device
        list when given (update_POI)."""
        self.fire.step(append_to)
        return self.fire.last_points()

    @property
    def grid(self) -> np.ndarray:
        return self.fire.grid()

    def run(self, iterations: int = num_iterations) -> list[np.ndarray]:
        """:76-86: export_data[0] = initial points, then one row per step."""
        for _ in range(iterations):
            self.export_data.append(self.update_grid())
        return self.export_data

    def close(self) -> None:
        self.fire.close()
