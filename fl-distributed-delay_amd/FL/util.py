"""Drop-in for the reference's FL/util.py (util.py:1-52), so `from FL.util import *`
(main.py:19) resolves to this package.

print_test_accuracy (util.py:31-45) runs the central model's forward on the MI355X engine
(flsim_<net>_eval_input: dropout off, BatchNorm from the running buffers) over the loader's
batches and returns the same scalar, 100 * correct / total.  The plotting helpers keep the
reference's behaviour (matplotlib is imported when they are called); check_mem reports device
memory through torch instead of shelling out to nvidia-smi (util.py:48-52), in the same
[total, used] MiB string form.
"""
import numpy as np
import torch


def save_data(x, y, savefile):
    """util.py:7-9."""
    print(np.stack([x, y]))
    np.save(savefile, np.stack([x, y]))


def plot_data(x, y, xlabel=None, ylabel=None, title=None, savefile=None):
    """util.py:12-21."""
    import matplotlib.pyplot as plt
    fig, ax = plt.subplots()
    ax.plot(x, y)
    ax.set(xlabel=xlabel, ylabel=ylabel, title=title)
    ax.grid()
    if savefile is not None:
        plt.savefig(savefile)


def imshow(img):
    """util.py:24-28."""
    import matplotlib.pyplot as plt
    img = img / 2 + 0.5     # unnormalize
    npimg = img.numpy()
    plt.imshow(np.transpose(npimg, (1, 2, 0)))
    plt.show()


def print_test_accuracy(model, testloader):
    """util.py:31-45: top-1 accuracy (%) of `model` over `testloader` (batches of
    (images NCHW float, labels)), predictions = first maximum of the logits.

    The device forward is the eval-mode one (dropout off, BatchNorm from the running buffers),
    which is how main.py:190 calls it (central.model.eval() first).  The reference would run
    model(images) in train mode too (random dropout masks, batch statistics); that is refused
    here rather than silently evaluated in eval mode."""
    from FL.agents import _context
    if model.training:
        raise NotImplementedError("print_test_accuracy on the HIP engine evaluates in eval mode: "
                                  "call model.eval() first (main.py:190)")
    ctx = _context(model)
    ctx.flush_backward()       # the evaluation reuses the workspace of deferred fwd_bkwd rows
    correct = 0
    total = 0
    with torch.no_grad():
        for data in testloader:
            images, labels = data
            pred = ctx.engine.evaluate_input(ctx.theta, images.to(ctx.device))
            labels = labels.to(ctx.device)
            total += labels.size(0)
            correct += (pred.to(labels.dtype) == labels).sum().item()
    print('Accuracy of the network on the 10000 test images: %d %%' % (
          100 * correct / total))
    return 100 * correct / total


def check_mem():
    """util.py:48-52 without nvidia-smi: [total MiB, used MiB] of the current device, as the
    strings the reference's CSV split returns."""
    free, total = torch.cuda.mem_get_info()
    return [str(total // 2 ** 20), " " + str((total - free) // 2 ** 20) + "\n"]
