from .mlp import MLPClassifier, WeatherClassifier, build_mlp  # noqa: F401
