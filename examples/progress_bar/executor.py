import time

from mlcomp_amd.worker.executors import Executor


@Executor.register
class Progress(Executor):
    def work(self):
        for _ in self.tqdm(list(range(300)), interval=1):
            time.sleep(0.01)
        return {}
