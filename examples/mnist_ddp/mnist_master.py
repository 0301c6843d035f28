"""Master for the MNIST examples: python mnist_master.py [--port 48148]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from pccl_amd.master import main  # noqa: E402

if __name__ == "__main__":
    main()
