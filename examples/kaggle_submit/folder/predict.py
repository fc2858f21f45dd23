"""Kernel entry point uploaded by `mlcomp submit`: load the traced model and write
submission.csv for the competition's test files."""
import glob

import pandas as pd
import torch


def main():
    model = torch.jit.load('net.pth').eval()
    rows = []
    for path in sorted(glob.glob('../input/test/*.pt')):
        with torch.no_grad():
            rows.append((path.split('/')[-1], float(torch.sigmoid(model(torch.load(path, weights_only=True))).mean())))
    pd.DataFrame(rows, columns=['filename', 'label']).to_csv('submission.csv', index=False)


if __name__ == '__main__':
    main()
