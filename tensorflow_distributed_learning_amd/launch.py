"""``python -m tensorflow_distributed_learning_amd.launch`` – see parallel/launch.py."""
import sys

from .parallel.launch import main

if __name__ == "__main__":
    sys.exit(main())
