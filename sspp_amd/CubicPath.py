"""Single-via cubic path — drop-in for the reference's ``sspp/CubicPath.py`` (lines 3-60).

p(u) = a u^3 + b u^2 + c u + d through start (u=0), via (u=0.5) and end (u=1) with zero
start velocity: a = 2 (end + 3 start - 4 via), b = 4 (via - start - a/8), c = 0, d = start.
u is clipped to [0, 1] before evaluation, as in the reference.
"""
import numpy as np


class CubicPath:
    def __init__(self):
        self.coefficients = None

    def plan(self, start, via, end):
        start, via, end = np.array(start), np.array(via), np.array(end)
        self.a = 2 * (end + 3 * start - 4 * via)
        self.b = 4 * (via - start - self.a / 8)
        self.c = 0
        self.d = start
        self.coefficients = (self.a, self.b, self.c, self.d)
        return True

    def evaluate(self, u):
        u = np.clip(u, 0, 1)
        return self.a * u ** 3 + self.b * u ** 2 + self.c * u + self.d

    def evaluate_with_derivatives(self, u):
        u = np.clip(u, 0, 1)
        pos = self.a * u ** 3 + self.b * u ** 2 + self.c * u + self.d
        vel = 3 * self.a * u ** 2 + 2 * self.b * u + self.c
        acc = 6 * self.a * u + 2 * self.b
        return pos, vel, acc
