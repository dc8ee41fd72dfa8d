class SchedulerMixin:
    """diffusers SchedulerMixin: only a base class on the training path."""
