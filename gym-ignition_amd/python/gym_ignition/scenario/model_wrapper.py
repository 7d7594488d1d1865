"""Delegating wrapper: unknown attributes resolve on the wrapped ScenarI/O model
(reference behaviour: python/gym_ignition/scenario/model_wrapper.py:9-20)."""


class ModelWrapper:
    def __init__(self, model):
        self.model = model

    def __getattr__(self, item):
        if item == "model":
            raise AttributeError(item)
        return getattr(self.model, item)
