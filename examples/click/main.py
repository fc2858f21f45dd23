import time

import click
from tqdm import tqdm


@click.group()
def base():
    pass


@base.command()
@click.option('--count', type=int, default=100)
def work(count: int):
    print('start')
    bar = tqdm(list(range(count)))
    for item in bar:
        bar.set_description(f'item={item}')
        time.sleep(0.01)
    print('end')


if __name__ == '__main__':
    base()
