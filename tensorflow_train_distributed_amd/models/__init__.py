"""Model zoo: the reference's MNIST MLP, ResNet-50 v1.5 and BERT (north-star models)."""
from .mlp import MLP, mnist_mlp
from .resnet import ResNet, resnet50
