import os

import torch


def device() -> torch.device:
    d = os.environ.get("MFA_DEVICE")
    if d:
        return torch.device(d)
    return torch.device("cuda:0" if torch.cuda.is_available() else "cpu")


def verbose() -> bool:
    return os.environ.get("MFA_VERBOSE", "0") not in ("0", "", "false")
