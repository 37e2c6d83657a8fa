from .mlp import MLPClassifier, WeatherClassifier, build_mlp  # noqa: F401


def build_model(name: str, input_dim: int, lr=None, **kw):
    """Model registry: ``weather`` (reference), MLP presets (``weather-mlp-3x128``,
    ``tabular-mlp-4x1024``) and ``tabtransformer`` (BASELINE config 5)."""
    if name.startswith("tabtransformer"):
        from .tabtransformer import TabTransformer

        args = dict(num_features=input_dim)
        if lr is not None:
            args["lr"] = lr
        args.update(kw)
        return TabTransformer(**args)
    return build_mlp(name, input_dim, **({} if lr is None else {"lr": lr}), **kw)
