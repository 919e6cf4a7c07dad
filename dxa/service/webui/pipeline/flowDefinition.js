// Flow definition panel (datax-pipeline flowDefinition/components/flowDefinitionPanel.jsx + flowActions.js):
// vertical tabs Info / Input / Reference data / Functions / Query / Rules / Outputs / Scale / Schedule over the
// designer model of one flow; Save, Deploy, Stop, Delete. Load = flow/get -> designer/flow/fromconfig; save =
// designer/flow/toconfig -> flow/save; deploy = save -> flow/startjobs (config generation runs server-side).
import { h, mount } from '../common/dom.js';
import { flowApi, servicePost, Constants } from '../common/api.js';
import { PageHeader, MessageBar, Spinner, Button, VerticalTabs, confirmDialog, functionEnabled, userContext } from '../common/components.js';
import * as Models from './models.js';
import { TAB_VALIDATORS, validateFlow } from './validation.js';
import { InfoTab, ReferenceDataTab, FunctionsTab, ScaleTab, ScheduleTab } from './tabs.js';
import { InputTab } from './inputTab.js';
import { RulesTab } from './rulesTab.js';
import { OutputsTab } from './outputsTab.js';
import { QueryTab } from '../query/index.js';

export const TABS = [
    ['info', 'Info', InfoTab],
    ['input', 'Input', InputTab],
    ['referenceData', 'Reference data', ReferenceDataTab],
    ['functions', 'Functions', FunctionsTab],
    ['query', 'Query', QueryTab],
    ['rules', 'Rules', RulesTab],
    ['outputs', 'Outputs', OutputsTab],
    ['scale', 'Scale', ScaleTab],
    ['schedule', 'Schedule', ScheduleTab]
];

export async function loadFlow(name) {
    const stored = await flowApi.get(name);
    const config = Object.assign({ name: stored.name, displayName: stored.displayName }, stored.gui || {});
    const flow = await servicePost(Constants.services.flow, 'designer/flow/fromconfig', { config });
    flow.name = flow.name || stored.name;
    flow.displayName = flow.displayName || stored.displayName || stored.name;
    return Models.normalizeFlow(flow);
}

export async function saveFlow(flow) {
    const config = await flowApi.toConfig(flow, flow.query);
    config.name = flow.name || undefined;
    return flowApi.save(config);
}

export function FlowDefinitionPanel(props, ctx) {
    const ui = {
        flow: null,
        tab: 'info',
        dirty: false,
        busy: null,
        message: null,
        selected: { referenceData: 0, functions: 0, outputs: 0, rules: 0, batchList: 0, batchInputs: 0 },
        kernel: { id: null, results: null, error: null },
        isNew: !props.id
    };
    const root = h('div');
    let navHost = null;
    let validity = {};

    ui.update = () => render();
    // a field changed: remember it and refresh the validity markers without rebuilding the editor under the cursor
    ui.touch = () => {
        ui.dirty = true;
        refreshMarkers();
    };
    ui.setMessage = (kind, text) => {
        ui.message = text ? { kind, text } : null;
        renderMessage();
    };

    function computeValidity() {
        const v = {};
        for (const [key] of TABS) v[key] = TAB_VALIDATORS[key] ? !!TAB_VALIDATORS[key](ui.flow) : true;
        return v;
    }

    function refreshMarkers() {
        validity = computeValidity();
        if (!navHost) return;
        for (const b of navHost.querySelectorAll('.vtab')) {
            const ok = validity[b.getAttribute('data-tab')];
            b.classList.toggle('invalid', !ok);
            let m = b.querySelector('.marker');
            if (!ok && !m) b.appendChild(h('span', { class: 'marker', title: 'incomplete settings' }, ' ●'));
            if (ok && m) m.remove();
        }
        const deploy = root.querySelector('button[data-act=deploy]');
        if (deploy) deploy.disabled = !functionEnabled('deployFlowButtonEnabled') || !validateFlow(ui.flow) || !!ui.busy;
        const title = root.querySelector('.page-header h2');
        if (title) title.textContent = (ui.flow.displayName || '(unnamed flow)') + (ui.dirty ? ' *' : '');
    }

    function renderMessage() {
        const host = root.querySelector('#flowmsg');
        if (host) mount(host, ui.message ? MessageBar(ui.message.kind, ui.message.text, () => ui.setMessage(null)) : null);
    }

    async function run(label, fn) {
        ui.busy = label;
        render();
        try {
            await fn();
        } catch (e) {
            ui.setMessage('error', `${label} failed: ${e.message}`);
        } finally {
            ui.busy = null;
            render();
        }
    }

    async function doSave() {
        const res = await saveFlow(ui.flow);
        const wasNew = !ui.flow.name;
        ui.flow.name = res.name;
        ui.dirty = false;
        ui.isNew = false;
        ui.setMessage('success', `Saved flow ${res.displayName || res.name}.`);
        if (wasNew) history.replaceState({}, '', `/config/edit/${res.name}`);
    }

    const actions = {
        save: () => run('Save', doSave),
        deploy: () =>
            run('Deploy', async () => {
                await doSave();
                await flowApi.generateConfigs(ui.flow.name);
                const jobs = await flowApi.startJobs(ui.flow.name);
                ui.setMessage('success', `Deployed ${ui.flow.name}: ${(jobs || []).map(j => (j && j.name ? `${j.name} ${j.state}` : String(j))).join(', ')}`);
            }),
        stop: () =>
            run('Stop', async () => {
                await flowApi.stopJobs(ui.flow.name);
                ui.setMessage('success', `Stopped the jobs of ${ui.flow.name}.`);
            }),
        remove: async () => {
            if (!(await confirmDialog('Delete flow', `Delete ${ui.flow.displayName}? Its jobs, runtime configs and checkpoints are removed.`))) return;
            await run('Delete', async () => {
                await flowApi.remove(ui.flow.name);
                ctx.navigate(props.returnPath || '/config');
            });
        }
    };

    function render() {
        if (!ui.flow) {
            mount(root, PageHeader('Flow'), h('div', { id: 'flowmsg' }), Spinner('Loading flow...'));
            renderMessage();
            return;
        }
        validity = computeValidity();
        const tabs = TABS.map(([key, label, Tab]) => ({ key, label, valid: validity[key], render: () => Tab(ui.flow, ui) }));
        const view = VerticalTabs(tabs, ui.tab, key => {
            ui.tab = key;
            render();
        });
        navHost = view.querySelector('.vtabs-nav');
        const saved = !!ui.flow.name;
        mount(
            root,
            PageHeader(
                (ui.flow.displayName || '(unnamed flow)') + (ui.dirty ? ' *' : ''),
                Button('Save', actions.save, { disabled: !functionEnabled('saveFlowButtonEnabled') || !!ui.busy }),
                h('button', {
                    class: 'primary',
                    'data-act': 'deploy',
                    disabled: !functionEnabled('deployFlowButtonEnabled') || !validateFlow(ui.flow) || !!ui.busy,
                    title: 'Save, generate the job config and start one process per GPU',
                    onclick: actions.deploy
                }, 'Deploy'),
                Button('Stop jobs', actions.stop, { disabled: !saved || !functionEnabled('jobActionsEnabled') || !!ui.busy }),
                Button('Delete', actions.remove, { disabled: !saved || !functionEnabled('deleteFlowButtonEnabled') || !!ui.busy }),
                Button('Back', () => ctx.navigate(props.returnPath || '/config'))
            ),
            h('div', { id: 'flowmsg' }),
            ui.busy ? Spinner(ui.busy + '...') : null,
            view
        );
        renderMessage();
    }

    (async () => {
        try {
            ui.flow = props.id ? await loadFlow(props.id) : Models.newFlow(userContext.enableLocalOneBox, userContext.user.name);
        } catch (e) {
            ui.flow = Models.newFlow(userContext.enableLocalOneBox, userContext.user.name);
            ui.setMessage('error', `Could not load flow ${props.id}: ${e.message}`);
        }
        render();
    })();
    render();
    ctx.onDispose(() => {
        if (ui.kernel.id) servicePost(Constants.services.interactiveQuery, 'kernel/delete', { kernelId: ui.kernel.id }).catch(() => null);
    });
    return root;
}

