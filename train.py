"""CLI twin of the reference launchers (src/single/main.py, src/ddp/main.py) on the native stack.

    python train.py single --epoch 50 --batch-size 128 --amp --contain-test
    python train.py ddp    --epoch 50 --batch-size 256 --amp --contain-test   # one process per GPU
"""
import sys

import dtc_import

if __name__ == "__main__":
    mode = sys.argv[1] if len(sys.argv) > 1 and sys.argv[1] in ("single", "ddp", "dp") else "ddp"
    argv = sys.argv[2:] if len(sys.argv) > 1 and sys.argv[1] == mode else sys.argv[1:]
    dtc_import.load().trainer.main(argv, mode)
