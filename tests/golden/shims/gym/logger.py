"""gym.logger stand-in (levels only)."""
DEBUG, INFO, WARN, ERROR, DISABLED = 10, 20, 30, 40, 50
_level = INFO


def set_level(level):
    global _level
    _level = level
