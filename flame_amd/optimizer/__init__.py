"""MI355X-native drop-ins for flame's server optimizers (lib/python/flame/optimizer/)."""
from .abstract import AbstractOptimizer
from .fedadagrad import FedAdaGrad
from .fedadam import FedAdam
from .fedavg import FedAvg
from .fedbuff import FedBuff
from .feddyn import FedDyn
from .fedgft import FedGFT
from .fedopt import FedOPT
from .fedprox import FedProx
from .fedyogi import FedYogi
from .scaffold import Scaffold
from .train_result import TrainResult

__all__ = ["AbstractOptimizer", "FedAvg", "FedOPT", "FedAdam", "FedYogi", "FedAdaGrad", "FedBuff",
           "FedProx", "FedDyn", "FedGFT", "Scaffold", "TrainResult"]
