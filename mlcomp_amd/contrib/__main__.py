"""``mlcomp-contrib``: k-fold split helpers writing ``fold.csv`` into the current folder
(`mlcomp/contrib/__main__.py:19-96`)."""
from __future__ import annotations

import os
import re
import uuid
from os.path import join

import click


def _grouper(regex):
    if not regex:
        return None
    pat = re.compile(regex)

    def get_group(x):
        m = pat.match(x)
        return m.group(1) if m else str(uuid.uuid4())
    return get_group


@click.group()
def main():
    pass


@main.command('split-pandas')
@click.argument('path')
@click.option('--n_splits', type=int, default=5)
def split_pandas(path, n_splits):
    import pandas as pd
    from mlcomp_amd.contrib.split import file_group_kfold
    df = pd.read_csv(path)
    folds = file_group_kfold(n_splits, image=list(df[df.columns[0]]))
    df['fold'] = folds['fold']   # index-aligned (the split shuffles rows)
    df.to_csv(join(os.getcwd(), 'fold.csv'), index=False)


@main.command('split-classify')
@click.argument('img_path')
@click.option('--n_splits', type=int, default=5)
@click.option('--group-regex')
def split_classify(img_path, n_splits, group_regex):
    from mlcomp_amd.contrib.split import file_group_kfold
    pairs = [(img, sub) for sub in sorted(os.listdir(img_path)) if os.path.isdir(join(img_path, sub))
             for img in sorted(os.listdir(join(img_path, sub)))]
    file_group_kfold(n_splits, join(os.getcwd(), 'fold.csv'), get_group=_grouper(group_regex),
                     image=[join(lab, img) for img, lab in pairs], label=[lab for _, lab in pairs])


@main.command('split-segment')
@click.argument('img_path')
@click.argument('mask_path')
@click.option('--n_splits', type=int, default=5)
@click.option('--group-regex')
def split_segment(img_path, mask_path, n_splits, group_regex):
    from mlcomp_amd.contrib.split import file_group_kfold
    file_group_kfold(n_splits, join(os.getcwd(), 'fold.csv'), get_group=_grouper(group_regex),
                     image=os.listdir(img_path), mask=os.listdir(mask_path), sort=True,
                     must_equal=['image', 'mask'])


@main.command('split-test-img')
@click.argument('img_path')
def split_test_img(img_path):
    import pandas as pd
    pd.DataFrame({'image': sorted(os.listdir(img_path)), 'fold': 0}).to_csv(
        join(os.getcwd(), 'fold_test.csv'), index=False)


@main.command('pack-records')
@click.argument('img_path')
@click.argument('out')
@click.option('--size', type=int, default=256, help='stored square size (shorter side resized, centre crop)')
@click.option('--fold-csv', default=None, help='fold.csv (image,label,fold): pack the rows of --fold only')
@click.option('--fold', type=int, default=None)
@click.option('--exclude-fold', is_flag=True, help='pack every fold except --fold (the training split)')
def pack_records(img_path, out, size, fold_csv, fold, exclude_fold):
    """Pack a class-per-folder image tree (or the rows of a fold.csv) into an .mlrec record
    file for the native input pipeline (mlcomp_amd.train.records)."""
    from mlcomp_amd.train.records import pack_images
    if fold_csv:
        import pandas as pd
        df = pd.read_csv(fold_csv)
        if fold is not None:
            df = df[(df['fold'] != fold) if exclude_fold else (df['fold'] == fold)]
        names = sorted(df['label'].astype(str).unique())
        paths = [join(img_path, p) for p in df['image']]
        labels = [names.index(str(v)) for v in df['label']]
    else:
        names = sorted(d for d in os.listdir(img_path) if os.path.isdir(join(img_path, d)))
        pairs = [(join(img_path, d, f), i) for i, d in enumerate(names) for f in sorted(os.listdir(join(img_path, d)))]
        paths, labels = [p for p, _ in pairs], [lab for _, lab in pairs]
    n = pack_images(paths, labels, out, size=size)
    with open(out + '.classes', 'w') as f:
        f.write('\n'.join(names) + '\n')
    click.echo(f'{n} images, {len(names)} classes -> {out}')


if __name__ == '__main__':
    main()
