from .cannet import (CANNet, make_layers, cannet_forward_reference, strip_module_prefix,  # noqa: F401
                     reference_state_dict_keys, CONTEXT_SCALES, FRONTEND_CFG, BACKEND_CFG)
