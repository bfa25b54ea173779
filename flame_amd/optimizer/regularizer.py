"""Server-side optimizers expose ``.regularizer`` because trainers instantiate the
optimizer only to read it (lib/python/flame/mode/horizontal/syncfl/trainer.py:74-77).

When the reference SDK is importable its own dummy Regularizer
(optimizer/regularizer/default.py) is used; otherwise an equivalent no-op.
"""
try:  # pragma: no cover - depends on flame being installed
    from flame.optimizer.regularizer.default import Regularizer  # type: ignore
except Exception:  # noqa: BLE001
    class Regularizer:
        """No-op regularizer (same methods as flame's default Regularizer)."""

        def get_term(self, **kwargs):
            return 0.0

        def save_state(self, state, **kwargs):
            pass

        def update(self):
            pass
