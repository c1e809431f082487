"""gym.wrappers stand-in: `Monitor` is only named by the reference's demo code paths."""


class Monitor:
    def __init__(self, *a, **k):
        raise RuntimeError("gym.wrappers.Monitor is not available in the offline harness")
