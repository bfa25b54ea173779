"""TrainResult -- lib/python/flame/optimizer/train_result.py:19-26 (weights, count, version)."""


class TrainResult(object):
    """Training result of one trainer and its metadata."""

    def __init__(self, weights=None, count=0, version=0):
        self.weights = weights
        self.count = count
        self.version = version
