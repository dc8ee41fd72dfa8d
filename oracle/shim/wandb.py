def init(*args, **kwargs):
    return None


def log(*args, **kwargs):
    return None


def finish(*args, **kwargs):
    return None
