"""Model families: the reference MNIST CNN (flagship, fused HIP path) and ResNet-50."""
