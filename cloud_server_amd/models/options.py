"""UI option catalog — apps/construction/util/options.py:4-58 (served by POST
/construct/options/).  Display strings are kept verbatim (they are what the front end
shows); ``DSL_TOKENS`` maps each display string to the DSL value the training config
uses, which the reference left to the front end."""
from __future__ import annotations

CATALOG = {
    "neural_network_type": {"options": ["传统神经网络", "CNN"], "default": "CNN"},
    "loss_function": {"options": ["平方差函数", "交叉熵函数"], "default": "平方差函数"},
    "optimizer": {"options": ["Gradient Descent Optimizer", "Adadelta Optimizer",
                              "Adagrad Optimizer", "Adam Optimizer"],
                  "default": "Gradient Descent Optimizer"},
    "param_init": {"options": ["全零", "正态分布", "Xavier"], "default": "全零"},
    "activation_method": {"options": ["Sigmoid", "ReLU"], "default": "ReLU"},
    "padding_method": {"options": ["SAME", "VALID"], "default": "SAME"},
}

DSL_TOKENS = {
    "传统神经网络": "DNN", "CNN": "CNN",
    "平方差函数": "mse", "交叉熵函数": "entropy",
    "Gradient Descent Optimizer": "GradientDescentOptimizer",
    "Adadelta Optimizer": "AdadeltaOptimizer",
    "Adagrad Optimizer": "AdagradOptimizer",
    "Adam Optimizer": "AdamOptimizer",
    "全零": "zero", "正态分布": "norm", "Xavier": "xavier",
    "Sigmoid": "sigmoid", "ReLU": "relu",
    "SAME": "SAME", "VALID": "VALID",
}


def get_options(name: str):
    if name not in CATALOG:
        raise KeyError(name)
    return dict(CATALOG[name], tokens={o: DSL_TOKENS[o] for o in CATALOG[name]["options"]})
