"""Closed value range [start, end] (reference struct/Clipping.py:1-17).

Clipping(abs=a) is the symmetric range [-|a|, |a|]; otherwise both start and end are required."""


class Clipping:
    def __init__(self, abs: float = None, start: float = None, end: float = None):
        if abs is None and (start is None or end is None):
            raise ValueError("Either abs or both start and end must be provided")
        if abs is None:
            self.start, self.end = start, end
        else:
            mag = abs if abs >= 0 else -abs
            self.start, self.end = -mag, mag
