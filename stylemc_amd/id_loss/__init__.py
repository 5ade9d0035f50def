from .id_loss import IDLoss  # noqa: F401
from .model_irse import Backbone, build_irse50  # noqa: F401
