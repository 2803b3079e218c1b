"""Inclusive index range shared by Puncture and Shortening."""


class InclusiveRange:
    _what = "range"

    def __init__(self, start: int, end: int):
        if start < 0 or end < 0 or start > end:
            raise ValueError(f"Invalid {self._what} range")
        self.start = start
        self.end = end
        self._len = end - start + 1

    def __len__(self):
        # note: Puncture(0, 0) has length 1, which enters the datagen's code rate
        return self._len
