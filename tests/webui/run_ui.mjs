// Drives the website's packages under node against a live control plane (tests/test_webui.py starts it and passes
// its base URL and a flow name with pre-loaded metrics). Prints one JSON line of observations per check.
import { installDom, waitFor, sleep, buttonByText } from './dom_shim.mjs';

const base = process.argv[2];
const metricFlow = process.argv[3];
const root = process.argv[4];
installDom(base);

const W = `${root}/dxa/service/webui`;
const out = {};
const ctx = extra => {
    const c = { navigate: p => (out.navigated = p), params: {}, disposers: [] };
    c.onDispose = fn => c.disposers.push(fn);
    return Object.assign(c, extra || {});
};

async function main() {
    const api = await import(`${W}/common/api.js`);
    const comps = await import(`${W}/common/components.js`);
    const app = await import(`${W}/app.js`);
    const Models = await import(`${W}/pipeline/models.js`);
    const V = await import(`${W}/pipeline/validation.js`);

    // ---- node server endpoints + user context
    const comp = await api.nodeGet('web-composition');
    out.pages = comp.pages.map(p => p.routePath);
    const route = app.resolvePage(comp.pages, '/config/edit/abc');
    out.route_edit = [route.page.componentName, route.params.id];
    out.route_new = app.resolvePage(comp.pages, '/config/new').page.componentName;
    comps.userContext.user = await api.nodeGet('user');
    comps.userContext.functions = await api.nodeGet('functionenabled');
    comps.userContext.enableLocalOneBox = (await api.nodeGet('enableLocalOneBox')).enableLocalOneBox;
    out.user = comps.userContext.user;
    out.n_functions = Object.keys(comps.userContext.functions).length;

    // ---- validation model
    const onebox = Models.newFlow(true, 'me');
    out.valid_onebox = V.validateFlow(onebox);
    const eh = Models.newFlow(false, 'me');
    out.valid_eventhub_noconn = V.validateInput(eh);
    eh.input.properties.inputEventhubConnection = 'Endpoint=sb://x/;EntityPath=y';
    out.valid_eventhub_conn = V.validateInput(eh);
    out.cond_err = V.conditionsError({ type: 'group', conditions: [{ type: 'condition', field: 't', operator: 'greater', value: 'abc' }] }, 'SimpleRule');

    // ---- flow list (empty), then a new flow through the definition panel
    const { FlowListPanel } = await import(`${W}/pipeline/flowList.js`);
    const list = FlowListPanel({ newItemPath: '/config/new', editItemPath: '/config/edit' }, ctx());
    document.body.appendChild(list);
    await waitFor(() => !list.textContent.includes('Loading flows'));
    out.list_before = list.textContent.includes('No flows yet');
    list.remove();

    const { FlowDefinitionPanel, loadFlow } = await import(`${W}/pipeline/flowDefinition.js`);
    const panel = FlowDefinitionPanel({ returnPath: '/config' }, ctx());
    document.body.appendChild(panel);
    await waitFor(() => panel.querySelector('.vtabs'));
    out.tabs = panel.querySelectorAll('.vtab').map(b => b.getAttribute('data-tab'));
    out.deploy_enabled_new = !panel.querySelector('button[data-act=deploy]').disabled;
    // Info tab: rename, then the Input tab: switch to Kafka -> the Input tab gets an incomplete marker
    const nameBox = panel.querySelector('.vtabs-body input');
    nameBox.input('UI Flow 1');
    buttonByText(panel, 'Input').click();
    const typeSel = panel.querySelectorAll('.vtabs-body select')[1];
    typeSel.input('kafka');
    await sleep(10);
    out.input_invalid_kafka = panel.querySelector('button[data-tab=input]').classList.contains('invalid');
    out.deploy_enabled_kafka = !panel.querySelector('button[data-act=deploy]').disabled;
    panel.querySelectorAll('.vtabs-body select')[1].input('local');
    await sleep(10);
    out.input_invalid_local = panel.querySelector('button[data-tab=input]').classList.contains('invalid');
    // Rules tab: add a rule, fill its condition; the preview comes from designer/conditions/sql
    buttonByText(panel, 'Rules').click();
    buttonByText(panel, '+ Add').click();
    const ruleInputs = () => panel.querySelectorAll('.vtabs-body .cond-group input');
    ruleInputs()[0].input('temperature');
    ruleInputs()[1].input('90');
    const desc = panel.querySelectorAll('.vtabs-body input').find(i => i.parentNode.textContent.startsWith('Description'));
    desc.input('too hot');
    const opSel = panel.querySelectorAll('.vtabs-body .cond-group select').find(s => s.querySelectorAll('option').some(o => o.value === 'greater'));
    opSel.input('greater');
    await waitFor(() => panel.textContent.includes('temperature > 90'), 3000);
    out.rule_preview = true;
    // Save: the name is derived from the display name
    buttonByText(panel, 'Save').click();
    await waitFor(() => panel.textContent.includes('Saved flow'), 5000);
    out.saved_path = location.pathname;
    const name = location.pathname.split('/').pop();
    const reloaded = await loadFlow(name);
    out.reloaded = { name: reloaded.name, type: reloaded.input.type, rules: reloaded.rules.length,
        cond: reloaded.rules[0].properties.conditions.conditions[0].field, display: reloaded.displayName };
    const stored = await api.flowApi.get(name);
    out.stored_condition = stored.gui.rules[0].properties.$condition;
    // Deploy generates the job config (starting it is left to the service test)
    await api.flowApi.generateConfigs(name);
    panel.remove();

    // ---- list again: the flow shows up with its job state
    const list2 = FlowListPanel({}, ctx());
    document.body.appendChild(list2);
    await waitFor(() => list2.querySelector('table'));
    out.list_after = list2.textContent.includes('UI Flow 1');
    list2.remove();

    // ---- jobs page
    const { GpuJobs } = await import(`${W}/jobs/index.js`);
    const c3 = ctx();
    const jobs = GpuJobs({}, c3);
    document.body.appendChild(jobs);
    await waitFor(() => jobs.querySelector('table'));
    out.jobs_row = jobs.textContent.includes(name);
    c3.disposers.forEach(f => f());
    jobs.remove();

    // ---- metrics: dashboard of a flow with pre-loaded points
    const M = await import(`${W}/metrics/index.js`);
    const f = await api.flowApi.get(metricFlow);
    const dash = M.Dashboard(f, { intervalMs: 60000 });
    document.body.appendChild(dash.root);
    await waitFor(() => dash.root.textContent.includes('6,000'), 5000);
    out.dash_text = dash.root.textContent.slice(0, 300);
    out.dash_svg_paths = dash.root.querySelectorAll('path').length;
    dash.stop();
    dash.root.remove();

    // ---- home page summary
    const { HomePage } = await import(`${W}/home/index.js`);
    const home = HomePage({}, ctx());
    document.body.appendChild(home);
    await waitFor(() => home.textContent.includes('Jobs running'), 5000);
    out.home = home.textContent.includes('UI Flow 1');
    console.log(JSON.stringify(out));
    process.exit(0);
}

main().catch(e => {
    console.log(JSON.stringify(Object.assign(out, { error: String(e && e.stack ? e.stack : e) })));
    process.exit(1);
});
