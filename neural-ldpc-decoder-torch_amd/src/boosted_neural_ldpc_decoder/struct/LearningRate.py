"""Step-decayed learning rate (reference struct/LearningRate.py:1-27).

Each call returns the current rate; every `decay_steps` calls the rate is multiplied by
`decay_rate`.  decay_rate == 0 or decay_steps <= 0 means a constant rate."""


class LearningRate:
    def __init__(self, initial_lr: float, decay_rate: float, decay_steps: int):
        self.lr = initial_lr
        self.decay_rate = decay_rate
        self.decay_steps = decay_steps
        self._calls = 0

    def __call__(self) -> float:
        if self.decay_rate == 0 or self.decay_steps <= 0:
            return self.lr
        current = self.lr
        self._calls += 1
        if self._calls >= self.decay_steps:
            self.lr *= self.decay_rate
            self._calls = 0
        return current
